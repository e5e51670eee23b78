#!/bin/bash
# Headline bench (N=65536) and a rocprofv3 kernel trace of the same command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_scaled.py -x -q --timeout 300 --timeout-method thread -k large > gpurun_out/t_large.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o r01 --output-format csv -- python3 bench.py --no-cpu > gpurun_out/prof.log 2>&1
rc=$?
echo "rc=$rc"
tail -n 3 gpurun_out/t_large.log; cat gpurun_out/bench.log; tail -n 5 gpurun_out/prof.log
exit $rc
