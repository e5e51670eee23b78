#!/bin/bash
# Interleaved A/B/... of S-C bench runs over prebuilt libraries (build_dbg/<name>/libgm.so),
# three rounds. usage: scripts/r06/ab_multi.sh <tag> <name> [<name> ...]   (no parity tests)
# SCEN=S-A|S-B|S-C (default S-C); STUB=1 adds the S-A stub-shard profile (shard_profile.py) per run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:?tag}; shift
O=gpurun_out/$T
mkdir -p $O
B="python3 bench.py --scenario ${SCEN:-S-C} --no-cpu --no-pmc --no-companion --steps ${STEPS:-10} --warmup 2"
for i in 1 2 3; do
  for n in "$@"; do
    GM_AB_BUILD=1 GM_LIBRARY=build_dbg/$n/libgm.so timeout -k 10 200 $B > $O/${n}_$i.json 2>/dev/null || exit 1
    if [ "${STUB:-0}" = 1 ]; then
      GM_AB_BUILD=1 GM_LIBRARY=build_dbg/$n/libgm.so timeout -k 10 200 python3 scripts/shard_profile.py --sb --cluster 65536 \
        > $O/${n}_stub_$i.json 2>/dev/null || exit 1
    fi
  done
done
for n in "$@"; do for f in $O/${n}_[0-9].json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3))"; done; done
if [ "${STUB:-0}" = 1 ]; then for n in "$@"; do for f in $O/${n}_stub_*.json; do echo "$f $(cut -c1-200 $f)"; done; done; fi
