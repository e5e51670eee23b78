#!/bin/bash
# Round 6 closing gate, part B: profiles of the final tree -- the S-A / S-B stub shards, the G = 8
# pipelined S-A and S-B loopbacks, the S-C row-shard loopback (+ rocprof stats), rocprof stats of S-A
# and S-C, per-tick S-A times, the SQ mixes of S-A and S-C.
# usage: scripts/r06/gate_close_b.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:?tag}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python3 scripts/shard_profile.py --sb > $O/sb_stub.json 2> $O/sb_stub.err || exit 1
timeout -k 10 300 python3 scripts/shard_profile.py --sb --cluster 65536 > $O/sa_stub.json 2> $O/sa_stub.err || exit 1
timeout -k 10 600 python3 scripts/sb_loopback_profile.py --pipelined > $O/sb_loopback_pipe.json 2> $O/sb_loopback_pipe.err || exit 1
timeout -k 10 300 python3 scripts/sb_loopback_profile.py --pipelined --cluster 65536 > $O/sa_loopback_pipe.json 2> $O/sa_loopback_pipe.err || exit 1
timeout -k 10 300 python3 scripts/partial_shard_profile.py > $O/pshard.json 2> $O/pshard.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_pshard -o ps -- python3 scripts/partial_shard_profile.py --ticks 6 > $O/prof_pshard.log 2>&1 || exit 1
bash scripts/gpu.sh $TAG prof_sa ticks prof_sc mix_sa mix_sc || exit 1
for f in $O/sb_stub.json $O/sa_stub.json $O/sb_loopback_pipe.json $O/sa_loopback_pipe.json $O/pshard.json; do cut -c1-300 $f; done
