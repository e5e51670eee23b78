#!/bin/bash
# round 5: gm_s_pick0 resolving every draw of a row at once (lane q: output q; one global round trip)
# -- SCALED / band-fast / msgcount / baseline-config tests on the tree, then the S-A bench (three
# interleaved rounds) and the S-B bench (one each): tree against var_q/libgm_head.so (the last commit).
#   usage: ab14.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05zc}
mkdir -p $O
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PT tests/test_gpu_scaled.py tests/test_gpu_band_fast.py tests/test_gpu_msgcount.py tests/test_gpu_baseline_configs.py tests/test_gpu_limits.py -m gpu > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
for k in 1 2 3; do
  timeout -k 10 300 python3 bench.py --no-cpu --no-pmc --no-companion > $O/sa_tree_$k.json 2> $O/sa_tree_$k.err || exit 1
  GM_AB_BUILD=1 GM_LIBRARY=var_q/libgm_head.so timeout -k 10 300 python3 bench.py --no-cpu --no-pmc --no-companion > $O/sa_head_$k.json 2> $O/sa_head_$k.err || exit 1
done
timeout -k 10 400 python3 bench.py --cluster 262144 --no-cpu --no-pmc > $O/sb_tree.json 2> $O/sb_tree.err || exit 1
GM_AB_BUILD=1 GM_LIBRARY=var_q/libgm_head.so timeout -k 10 400 python3 bench.py --cluster 262144 --no-cpu --no-pmc > $O/sb_head.json 2> $O/sb_head.err || exit 1
for f in $O/s?_*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f', round(d['roofline']['kernel_ms'],3), round(d['ms_per_step'],3), round(d['ms_per_step']-d['roofline']['kernel_ms'],3), round(d['value']/1e6,2))"; done
