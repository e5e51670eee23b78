#!/bin/bash
# round-4 experiment: gm_s_pick / gm_s_draw occupancy hints (measurement builds varlib/pick6, pick8)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04t
mkdir -p $O
for v in main pick6 pick8; do
  L=distributed-membership_amd/lib/libgm.so; [ $v != main ] && L=varlib/$v/libgm.so
  GM_AB_BUILD=1 GM_LIBRARY=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o p -- \
    python3 bench.py --no-cpu --no-pmc --no-companion > $O/bench_$v.json 2> $O/bench_$v.err || exit 1
done
