#!/bin/bash
# Banded tick: SCALED + sharded parity, then bench A/B over band widths.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_scaled.py tests/test_gpu_sharded.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_scaled.log 2>&1 &&
timeout -k 10 200 python -u bench.py --no-cpu > gpurun_out/bench_auto.log 2>&1 &&
GM_BAND=64 timeout -k 10 200 python -u bench.py --no-cpu > gpurun_out/bench_b64.log 2>&1 &&
GM_BAND=256 timeout -k 10 200 python -u bench.py --no-cpu > gpurun_out/bench_b256.log 2>&1 &&
GM_BAND=512 timeout -k 10 200 python -u bench.py --no-cpu > gpurun_out/bench_b512.log 2>&1
rc=$?
echo "rc=$rc"; grep -E "passed|failed|Error|error" gpurun_out/t_scaled.log | tail -5
for f in auto b64 b256 b512; do python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_$f.log').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])" 2>/dev/null || tail -3 gpurun_out/bench_$f.log; done
exit $rc
