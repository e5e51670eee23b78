#!/bin/bash
# rocprofv3 kernel stats of the S-A stub shard (rank 3 of 8, 8,192 columns) for each prebuilt
# library build_dbg/<name>/libgm.so. usage: scripts/r06/prof_stub.sh <tag> <name> [<name> ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:?tag}; shift
O=gpurun_out/$T
mkdir -p $O
for n in "$@"; do
  GM_AB_BUILD=1 GM_LIBRARY=build_dbg/$n/libgm.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $O/prof_$n -o s -- python3 scripts/shard_profile.py --sb --cluster ${STUB_N:-65536} > $O/stub_$n.json 2> $O/stub_$n.err || exit 1
done
for n in "$@"; do echo "== $n $(cut -c1-160 $O/stub_$n.json)"; f=$(find $O/prof_$n -name '*kernel_stats.csv' | head -1); cut -d, -f1-4 "$f" | head -12; done
