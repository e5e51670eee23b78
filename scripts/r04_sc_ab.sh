#!/bin/bash
# round-4 A/B on one box: the S-C bench with the in-tree library (main) and with variant libraries
# varlib/NAME (VARS, default scprev = the previous gm_partial.hip), alternating, tick kernels by HIP events
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${AB_TAG:-r04ze}
mkdir -p $O
for i in 1 2; do
  for v in main ${VARS:-scprev}; do
    L=distributed-membership_amd/lib/libgm.so; [ $v != main ] && L=varlib/$v/libgm.so
    GM_AB_BUILD=1 GM_LIBRARY=$L timeout -k 10 300 python -u bench.py --scenario S-C --no-cpu --no-pmc --steps 10 --warmup 2 \
      > $O/sc_${v}_$i.json 2> $O/sc_${v}_$i.err || exit 1
  done
done
