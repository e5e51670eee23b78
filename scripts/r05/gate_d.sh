#!/bin/bash
# round 5: four-rows-per-wave draw round 0 -- shard tests, S-B stub (draw0 vs old), S-B G = 8 loopback
# (pipelined order and phase API), the fused S-B on the same box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05e}
mkdir -p $O
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PT tests/test_gpu_sharded.py tests/test_gpu_gloo_shards.py tests/test_gpu_msgcount.py \
  tests/test_gpu_fullsize_shards.py tests/test_gpu_limits.py -m gpu --durations 10 > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -3 $O/gpu_tests.txt
timeout -k 10 300 python3 scripts/shard_profile.py --sb > $O/sb_k4.json 2> $O/sb_k4.err &&
GM_DRAW0=0 timeout -k 10 300 python3 scripts/shard_profile.py --sb > $O/sb_k4_olddraw.json 2> $O/sb_k4_olddraw.err &&
GM_SHARD_PIPE=0 timeout -k 10 300 python3 scripts/shard_profile.py --sb > $O/sb_nopipe.json 2> $O/sb_nopipe.err &&
timeout -k 10 300 python3 scripts/shard_profile.py --sb --cluster 65536 > $O/sa_k4.json 2> $O/sa_k4.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sbshard -o s -- \
  python3 scripts/shard_profile.py --sb > $O/sb_prof.json 2> $O/sb_prof.err &&
timeout -k 10 600 python3 scripts/sb_loopback_profile.py --pipelined > $O/sb_loopback_pipe.json 2> $O/sb_loopback_pipe.err &&
timeout -k 10 600 python3 scripts/sb_loopback_profile.py > $O/sb_loopback_phase.json 2> $O/sb_loopback_phase.err &&
timeout -k 10 400 python3 bench.py --cluster 262144 --no-cpu --no-pmc > $O/bench_sb.json 2> $O/bench_sb.err
rc=$?
for f in $O/*.json; do echo "$f $(cut -c1-300 $f)"; done
exit $rc
