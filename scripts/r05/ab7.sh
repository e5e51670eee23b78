#!/bin/bash
# round 5: S-C list-load / merge steps past the node's lists skipped by a scalar branch (GM_P_SKIP) --
# PARTIAL parity on the tree, then the S-C bench of the tree against var_sc/libgm_skip0.so, interleaved.
#   usage: ab7.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05p}
mkdir -p $O
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PT tests/test_gpu_partial.py -m gpu > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
for k in 1 2 3; do
  timeout -k 10 300 python3 bench.py --scenario S-C --no-cpu --no-pmc --steps 10 --warmup 2 > $O/sc_tree_$k.json 2> $O/sc_tree_$k.err || exit 1
  GM_AB_BUILD=1 GM_LIBRARY=var_sc/libgm_skip0.so timeout -k 10 300 python3 bench.py --scenario S-C --no-cpu --no-pmc --steps 10 --warmup 2 > $O/sc_skip0_$k.json 2> $O/sc_skip0_$k.err || exit 1
done
for f in $O/sc_*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f', round(d['roofline']['kernel_ms'],3), round(d['ms_per_step'],3), round(d['value']/1e6,1))"; done
