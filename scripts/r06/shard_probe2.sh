#!/bin/bash
# The S-A stub shard after the stub-target fix (rank 3, 2 and 1 exchange chunks; rank 0), the S-B stub,
# and the real G = 8 pipelined loopback of S-A and S-B (every shard's kernels serialised on one device).
# usage: scripts/r06/shard_probe2.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
P="timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv"
$P -d $O/k2 -o s -- python3 scripts/shard_profile.py --sb --cluster 65536 > $O/sa_stub.json 2>$O/k2.err &&
GM_SCHUNKS=1 $P -d $O/k1 -o s -- python3 scripts/shard_profile.py --sb --cluster 65536 > $O/sa_stub_k1.json 2>$O/k1.err &&
$P -d $O/r0 -o s -- python3 scripts/shard_profile.py --sb --cluster 65536 --rank 0 > $O/sa_stub_r0.json 2>$O/r0.err &&
$P -d $O/sb -o s -- python3 scripts/shard_profile.py --sb > $O/sb_stub.json 2>$O/sb.err &&
timeout -k 10 300 python3 scripts/sb_loopback_profile.py --cluster 65536 --pipelined > $O/sa_loop.json 2>$O/sa_loop.err &&
timeout -k 10 400 python3 scripts/sb_loopback_profile.py --pipelined > $O/sb_loop.json 2>$O/sb_loop.err
rc=$?
echo rc=$rc
for f in $O/*.json; do echo "$f $(cut -c1-300 $f)"; done
exit $rc
