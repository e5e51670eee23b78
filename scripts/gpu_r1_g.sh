#!/bin/bash
# Re-entry check: GPU parity suite, default bench, selected-region rocprof trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --selected-regions --kernel-trace --stats -d gpurun_out/prof_sel -o r01 --output-format csv -- python3 bench.py --no-cpu > gpurun_out/prof_sel.log 2>&1
rc=$?
echo "rc=$rc"; tail -n 3 gpurun_out/t_all.log; cat gpurun_out/bench.log; cat gpurun_out/prof_sel/r01_kernel_stats.csv 2>/dev/null || find gpurun_out/prof_sel -name '*stats*'
exit $rc
