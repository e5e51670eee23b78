#!/bin/bash
# round 5: S-A (1) the tick's counters zeroed by gm_s_mtgen instead of two fill launches per tick
# (var_q/libgm_mt.so), (2) plus the fast path's row counts reduced once (the tree) -- SCALED / band-fast
# / shard / event tests on the tree, then three interleaved rounds of the S-A bench: tree, mt, head
# (the last commit).   usage: ab10.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05t}
mkdir -p $O
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PT tests/test_gpu_band_fast.py tests/test_gpu_scaled.py tests/test_gpu_sharded.py tests/test_gpu_limits.py tests/test_gpu_msgcount.py tests/test_gpu_ramp.py -m gpu > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
for k in 1 2 3; do
  timeout -k 10 300 python3 bench.py --no-cpu --no-pmc --no-companion > $O/sa_tree_$k.json 2> $O/sa_tree_$k.err || exit 1
  for v in mt head; do
    GM_AB_BUILD=1 GM_LIBRARY=var_q/libgm_$v.so timeout -k 10 300 python3 bench.py --no-cpu --no-pmc --no-companion > $O/sa_${v}_$k.json 2> $O/sa_${v}_$k.err || exit 1
  done
done
for f in $O/sa_*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f', round(d['roofline']['kernel_ms'],3), round(d['ms_per_step'],3), round(d['value']/1e6,2))"; done
