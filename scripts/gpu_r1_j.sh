#!/bin/bash
# narrow-cell band kernel: per-tick trace + SQ counters (one pass) at B=512.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
GM_BAND=512 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pj -o r --output-format csv -- python3 bench.py --no-cpu --steps 10 > gpurun_out/pj.log 2>&1 &&
GM_BAND=512 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY --kernel-trace --output-format csv -d gpurun_out/pjc -o r -- python3 bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/pjc.log 2>&1
rc=$?
echo "rc=$rc"
find gpurun_out/pj -name '*kernel_stats.csv' -exec cat {} \;
exit $rc
