#!/bin/bash
# S-C per-section attribution: measurement builds build_dbg/sc_l<level>/libgm.so
# (scripts/r06/sc_sections_variant.py + hipcc) cut the LAST tick (42) after section <level>; for each,
# a kernel-trace run (that tick's kernel time) and one SQ-mix pass (instructions per dispatch).
# usage: scripts/r06/sc_sections.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
CMD="python3 bench.py --scenario S-C --no-cpu --no-pmc --steps 16 --warmup 1"
for l in ${LEVELS:-1 2 3 4 5}; do
  L=build_dbg/sc_l$l/libgm.so
  GM_AB_BUILD=1 GM_LIBRARY=$L timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace_l$l -o sc -- \
    $CMD > $O/trace_l$l.log 2>&1 || exit 1
  GM_AB_BUILD=1 GM_LIBRARY=$L timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    --kernel-trace --output-format csv -d $O/mix_l$l -o p -- $CMD > $O/mix_l$l.log 2>&1 || exit 1
  echo "level $l done"
done
