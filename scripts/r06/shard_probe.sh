#!/bin/bash
# Why does a column shard's band kernel cost more per (row, band) unit than the fused kernel?
# (1) the S-A stub shard at 2 and 1 exchange chunks, rank 3 and rank 0; (2) the fused S-A tick forced
# through the one-rank RCCL sharded path (full width, pipelined, 2 chunks) -- kernel traces of each.
# usage: scripts/r06/shard_probe.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
P="timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv"
$P -d $O/k2 -o s -- python3 scripts/shard_profile.py --sb --cluster 65536 > $O/k2.json 2>&1 &&
GM_SCHUNKS=1 $P -d $O/k1 -o s -- python3 scripts/shard_profile.py --sb --cluster 65536 > $O/k1.json 2>&1 &&
$P -d $O/r0 -o s -- python3 scripts/shard_profile.py --sb --cluster 65536 --rank 0 > $O/r0.json 2>&1 &&
$P -d $O/g4 -o s -- python3 scripts/shard_profile.py --sb --cluster 65536 --shards 4 > $O/g4.json 2>&1 &&
$P -d $O/force -o s -- python3 bench.py --force-shard --no-cpu --no-pmc --no-companion > $O/force.json 2>&1 &&
$P -d $O/fused -o s -- python3 bench.py --no-cpu --no-pmc --no-companion > $O/fused.json 2>&1
rc=$?
echo rc=$rc
exit $rc
