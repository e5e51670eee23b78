#!/bin/bash
# round 5: the pipelined column-shard tick -- shard tests, then the S-B stub shard pipelined vs not
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05c}
mkdir -p $O
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PT tests/test_gpu_sharded.py tests/test_gpu_gloo_shards.py tests/test_gpu_msgcount.py \
  tests/test_gpu_band_fast.py tests/test_gpu_fullsize_shards.py -m gpu --durations 10 > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -3 $O/gpu_tests.txt
timeout -k 10 300 python3 scripts/shard_profile.py --sb > $O/sb_shard_pipe.json 2> $O/sb_shard_pipe.err &&
GM_SHARD_PIPE=0 timeout -k 10 300 python3 scripts/shard_profile.py --sb > $O/sb_shard_nopipe.json 2> $O/sb_shard_nopipe.err &&
timeout -k 10 300 python3 scripts/shard_profile.py --sb --cluster 65536 > $O/sa_shard_pipe.json 2> $O/sa_shard_pipe.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sbshard -o s -- \
  python3 scripts/shard_profile.py --sb > $O/sb_shard_prof.json 2> $O/sb_shard_prof.err
rc=$?
cat $O/*.json
exit $rc
