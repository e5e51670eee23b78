#!/bin/bash
# Round gate: full GPU suite with durations, smoke, default bench, S-C bench (+cpu baseline).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/z
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=12 > gpurun_out/z/t_all.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/z/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/z/bench.log 2>&1 &&
timeout -k 10 400 python -u bench.py --scenario S-C > gpurun_out/z/bench_sc.log 2>&1
rc=$?
echo "rc=$rc"; tail -n 16 gpurun_out/z/t_all.log; tail -n 1 gpurun_out/z/smoke.log; tail -n 1 gpurun_out/z/bench.log | cut -c1-200; tail -n 1 gpurun_out/z/bench_sc.log | cut -c1-200
exit $rc
