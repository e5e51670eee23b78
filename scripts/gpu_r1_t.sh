#!/bin/bash
# Row-shard RCCL single-rank rehearsal + S-C bench with the exchange forced on (and off).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/sc4
timeout -k 10 300 python -u -m pytest tests/test_gpu_partial.py -x -v --timeout 200 --timeout-method thread -k "rccl or row_shards" > gpurun_out/sc4/t.log 2>&1 &&
timeout -k 10 300 python -u bench.py --scenario S-C --no-cpu --force-shard > gpurun_out/sc4/bench_force.log 2>&1
rc=$?
echo "rc=$rc"; grep -E "PASS|FAIL|passed|failed|Error|assert" gpurun_out/sc4/t.log | tail -6; tail -n 1 gpurun_out/sc4/bench_force.log
exit $rc
