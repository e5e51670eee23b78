#!/bin/bash
# round 5: rocprof breakdown of ONE S-B column shard (and one S-A shard) alone on the device
# (gm_shard_stub), to split the per-tick non-band work by kernel
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05a}
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sbshard -o s -- \
  python3 scripts/shard_profile.py --sb > $O/sb_shard.json 2> $O/sb_shard.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sashard -o s -- \
  python3 scripts/shard_profile.py --sb --cluster 65536 > $O/sa_shard.json 2> $O/sa_shard.err
rc=$?
cat $O/sb_shard.json $O/sa_shard.json
exit $rc
