#!/bin/bash
# round 5: shard tests + S-B stub shard: pipelined (K = 4, 8) vs unpipelined, S-A stub, rocprof of the K = 4 run
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05d}
mkdir -p $O
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PT tests/test_gpu_sharded.py tests/test_gpu_gloo_shards.py tests/test_gpu_msgcount.py \
  tests/test_gpu_fullsize_shards.py -m gpu --durations 10 > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -3 $O/gpu_tests.txt
timeout -k 10 300 python3 scripts/shard_profile.py --sb > $O/sb_k4.json 2> $O/sb_k4.err &&
GM_SCHUNKS=8 timeout -k 10 300 python3 scripts/shard_profile.py --sb > $O/sb_k8.json 2> $O/sb_k8.err &&
GM_SHARD_PIPE=0 timeout -k 10 300 python3 scripts/shard_profile.py --sb > $O/sb_nopipe.json 2> $O/sb_nopipe.err &&
timeout -k 10 300 python3 scripts/shard_profile.py --sb --cluster 65536 > $O/sa_k4.json 2> $O/sa_k4.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sbshard -o s -- \
  python3 scripts/shard_profile.py --sb > $O/sb_prof.json 2> $O/sb_prof.err &&
GM_SHARD_PIPE=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sbshard_nopipe -o s -- \
  python3 scripts/shard_profile.py --sb > $O/sb_prof_nopipe.json 2> $O/sb_prof_nopipe.err
rc=$?
for f in $O/*.json; do echo "$f $(cut -c1-330 $f)"; done
exit $rc
