#!/bin/bash
# Interleaved A/B/... of S-C bench runs over prebuilt libraries (build_dbg/<name>/libgm.so),
# three rounds. usage: scripts/r06/ab_multi.sh <tag> <name> [<name> ...]   (no parity tests)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:?tag}; shift
O=gpurun_out/$T
mkdir -p $O
B="python3 bench.py --scenario ${SCEN:-S-C} --no-cpu --no-pmc --steps ${STEPS:-10} --warmup 2"
for i in 1 2 3; do
  for n in "$@"; do
    GM_AB_BUILD=1 GM_LIBRARY=build_dbg/$n/libgm.so timeout -k 10 200 $B > $O/${n}_$i.json 2>/dev/null || exit 1
  done
done
for n in "$@"; do for f in $O/${n}_*.json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3))"; done; done
