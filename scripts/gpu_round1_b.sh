#!/bin/bash
# Full GPU test suite, then the headline bench (N=65536) and a rocprofv3 kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o r01 -- python3 bench.py --no-cpu --steps 10 > gpurun_out/prof.log 2>&1
rc=$?
echo "rc=$rc"
tail -n 3 gpurun_out/t_all.log; cat gpurun_out/bench.log
exit $rc
