#!/bin/bash
# Round-1 measurement of the banded narrow-cell tick: default bench (with cpu_baseline),
# kernel trace + stats of the same command, PMC FETCH_SIZE / WRITE_SIZE passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 300 python -u bench.py > gpurun_out/prof/bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o band --output-format csv -- python3 bench.py --no-cpu > gpurun_out/prof/trace.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/prof/pmc_fetch -o band -- python3 bench.py --no-cpu --steps 8 --warmup 1 > gpurun_out/prof/pmc_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/prof/pmc_write -o band -- python3 bench.py --no-cpu --steps 8 --warmup 1 > gpurun_out/prof/pmc_write.log 2>&1
rc=$?
echo "rc=$rc"; cat gpurun_out/prof/bench.log | tail -1; find gpurun_out/prof/trace -name '*kernel_stats.csv' -exec cat {} \;
exit $rc
