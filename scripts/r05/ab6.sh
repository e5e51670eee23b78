#!/bin/bash
# round 5: row-shard gm_p_pack as one workgroup per tile for every peer (each node's list read and
# converted once) -- PARTIAL / row-shard parity, then the G = 8 loopback profile of the tree against
# var_fast/libgm_pack0.so (the per-peer pack), interleaved.   usage: ab6.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05n}
mkdir -p $O
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PT tests/test_gpu_partial.py tests/test_gpu_fullsize_shards.py tests/test_gpu_gloo_shards.py -m gpu > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
for k in 1 2; do
  timeout -k 10 300 python3 scripts/partial_shard_profile.py > $O/pshard_tree_$k.json 2> $O/pshard_tree_$k.err || exit 1
  GM_AB_BUILD=1 GM_LIBRARY=var_fast/libgm_pack0.so timeout -k 10 300 python3 scripts/partial_shard_profile.py > $O/pshard_pack0_$k.json 2> $O/pshard_pack0_$k.err || exit 1
done
for f in $O/pshard_*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f', round(d['ms_per_tick_all_shards_serialised']/d['shards'],3), d['recv_mb_mean'])"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_pshard -o ps -- python3 scripts/partial_shard_profile.py --ticks 6 > $O/prof_pshard.log 2>&1 || exit 1
f=$(ls $O/prof_pshard/*kernel_stats.csv | head -1); head -12 "$f" | cut -d, -f1-5
