#!/bin/bash
# round 5: (1) S-A band kernels, this tree (round-5 SState fields moved to the end, no unit bounds in
# the fused fast kernel) vs round 4's library, interleaved; (2) the S-C row-shard G = 8 loopback at 4 / 8 / 16
# nodes per wave in the chunk launches
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05k}
mkdir -p $O
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PT tests/test_gpu_scaled.py tests/test_gpu_band_fast.py tests/test_gpu_sharded.py tests/test_gpu_partial.py \
  tests/test_gpu_fullsize_shards.py -m gpu > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -3 $O/gpu_tests.txt
for k in 1 2 3; do
  timeout -k 10 300 python3 bench.py --no-cpu --no-pmc --no-companion > $O/sa_cur_$k.json 2> $O/sa_cur_$k.err || exit 1
  GM_AB_BUILD=1 GM_LIBRARY=var_ab/libgm_r04.so timeout -k 10 300 python3 bench.py --no-cpu --no-pmc --no-companion > $O/sa_r04_$k.json 2> $O/sa_r04_$k.err || exit 1
done
for f in $O/sa_*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f', round(d['roofline']['kernel_ms'],3), round(d['ms_per_step'],3), round(d['value']/1e6,2))"; done
timeout -k 10 300 python3 scripts/partial_shard_profile.py > $O/pshard_npw4.json 2> $O/pshard_npw4.err || exit 1
for v in 8 16; do
  GM_AB_BUILD=1 GM_LIBRARY=var_pshard/libgm_npw$v.so timeout -k 10 300 python3 scripts/partial_shard_profile.py > $O/pshard_npw$v.json 2> $O/pshard_npw$v.err || exit 1
done
for f in $O/pshard_*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f', round(d['ms_per_tick_all_shards_serialised']/d['shards'],3), d['recv_mb_mean'])"; done
