#!/bin/bash
# round 5: exchange chunks K = 1 / 2 for the S-A column shards (N = 65,536, G = 8): the stub shard and
# the pipelined G = 8 loopback.   usage: ab13.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05za}
mkdir -p $O
for k in 1 2; do
  for K in 1 2; do
    GM_SCHUNKS=$K timeout -k 10 300 python3 scripts/shard_profile.py --sb --cluster 65536 > $O/sa_stub_k${K}_$k.json 2> $O/sa_stub_k${K}_$k.err || exit 1
    GM_SCHUNKS=$K timeout -k 10 300 python3 scripts/sb_loopback_profile.py --pipelined --cluster 65536 > $O/sa_loop_k${K}_$k.json 2> $O/sa_loop_k${K}_$k.err || exit 1
  done
done
for f in $O/sa_stub_*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f', round(d['ms_per_tick'],3), round(d['band_kernel_ms'],3), round(d['other_kernels_ms'],3))"; done
for f in $O/sa_loop_*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f', round(d['ms_per_shard_tick'],3))"; done
