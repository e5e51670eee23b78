#!/bin/bash
# S-C per-section attribution (measurement build build_dbg/sc_sections/libgm.so, made by
# scripts/r06/sc_sections_variant.py + hipcc): a kernel-trace run (per-tick kernel time of the
# ablated ticks) and one SQ-mix pass (instructions per dispatch), same bench command.
# usage: scripts/r06/sc_sections.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
L=build_dbg/sc_sections/libgm.so
CMD="python3 bench.py --scenario S-C --no-cpu --no-pmc --steps 16 --warmup 1"
GM_AB_BUILD=1 GM_LIBRARY=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o sc -- \
  $CMD > $O/trace.log 2>&1 &&
GM_AB_BUILD=1 GM_LIBRARY=$L timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  --kernel-trace --output-format csv -d $O/mix -o p -- $CMD > $O/mix.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
