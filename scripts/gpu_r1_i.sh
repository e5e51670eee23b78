#!/bin/bash
# Banded tick: kernel trace at B=128/512 + PMC traffic at B=128.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
GM_BAND=128 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pb128 -o r --output-format csv -- python3 bench.py --no-cpu --steps 10 > gpurun_out/pb128.log 2>&1 &&
GM_BAND=512 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pb512 -o r --output-format csv -- python3 bench.py --no-cpu --steps 10 > gpurun_out/pb512.log 2>&1 &&
GM_BAND=128 timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmcf128 -o r -- python3 bench.py --no-cpu --steps 5 --warmup 1 > gpurun_out/pmcf128.log 2>&1 &&
GM_BAND=128 timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmcw128 -o r -- python3 bench.py --no-cpu --steps 5 --warmup 1 > gpurun_out/pmcw128.log 2>&1
rc=$?
echo "rc=$rc"
for d in pb128 pb512; do find gpurun_out/$d -name '*kernel_stats.csv' -exec cat {} \; ; done
exit $rc
