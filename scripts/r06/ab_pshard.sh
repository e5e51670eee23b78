#!/bin/bash
# Interleaved runs of the S-C G = 8 row-shard loopback (scripts/partial_shard_profile.py) over prebuilt
# libraries build_dbg/<name>/libgm.so. usage: scripts/r06/ab_pshard.sh <tag> <name> [<name> ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${1:?tag}; shift; mkdir -p $O
for i in 1 2; do
  for n in "$@"; do
    GM_AB_BUILD=1 GM_LIBRARY=build_dbg/$n/libgm.so timeout -k 10 300 python3 scripts/partial_shard_profile.py \
      > $O/${n}_$i.json 2> $O/${n}_$i.err || exit 1
  done
done
for n in "$@"; do for f in $O/${n}_[0-9].json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['ms_per_tick_all_shards_serialised']/d['shards'],3))"; done; done
