#!/bin/bash
# PARTIAL change check: PARTIAL parity tests (1 GPU + row shards), smoke, S-C bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/rank
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_partial.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --scenario S-C > $O/bench_sc.json 2> $O/bench_sc.err
rc=$?
echo "rc=$rc"; tail -n 2 $O/tests.txt; tail -n 1 $O/smoke.txt; cut -c1-260 $O/bench_sc.json
python3 -c "import json; d=json.load(open('$O/bench_sc.json')); print(round(d['ms_per_step'],2), round(d['roofline']['kernel_ms'],2))" || true
exit $rc
