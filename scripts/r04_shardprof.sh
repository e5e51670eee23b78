#!/bin/bash
# round-4: one column shard alone on the device (gm_shard_stub: the real kernels at the true shard
# shape, collectives replaced by local stand-ins), S-B (N = 262,144) and S-A (N = 65,536), G = 8
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04s
mkdir -p $O
timeout -k 10 300 python -u scripts/shard_profile.py --sb > $O/sb_shard.json 2> $O/sb_shard.err || exit 1
timeout -k 10 200 python -u scripts/shard_profile.py --sb --cluster 65536 > $O/sa_shard.json 2> $O/sa_shard.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sa_shard -o sa -- \
  python3 scripts/shard_profile.py --sb --cluster 65536 > $O/prof_sa_shard.log 2>&1 || exit 1
