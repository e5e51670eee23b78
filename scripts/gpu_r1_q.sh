#!/bin/bash
# PARTIAL rewrite (small/big table kernels): parity vs oracle, then S-C bench + kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/sc2
timeout -k 10 600 python -u -m pytest tests/test_gpu_partial.py -x -v --timeout 400 --timeout-method thread > gpurun_out/sc2/t_partial.log 2>&1 &&
timeout -k 10 300 python -u bench.py --scenario S-C --no-cpu > gpurun_out/sc2/bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sc2/trace -o sc --output-format csv -- python3 bench.py --scenario S-C --no-cpu --steps 10 > gpurun_out/sc2/trace.log 2>&1
rc=$?
echo "rc=$rc"; grep -E "passed|failed|Error|assert" gpurun_out/sc2/t_partial.log | tail -5; tail -n 1 gpurun_out/sc2/bench.log; find gpurun_out/sc2/trace -name '*kernel_stats.csv' -exec cat {} \;
exit $rc
