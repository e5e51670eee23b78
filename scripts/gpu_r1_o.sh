#!/bin/bash
# S-C (partial views, N = 16M) first measurement: bench line + kernel trace/stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/sc
timeout -k 10 400 python -u bench.py --scenario S-C > gpurun_out/sc/bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sc/trace -o sc --output-format csv -- python3 bench.py --scenario S-C --no-cpu --steps 10 > gpurun_out/sc/trace.log 2>&1
rc=$?
echo "rc=$rc"; tail -n 2 gpurun_out/sc/bench.log; find gpurun_out/sc/trace -name '*kernel_stats.csv' -exec cat {} \;
exit $rc
