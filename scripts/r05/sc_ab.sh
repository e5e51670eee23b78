#!/bin/bash
# round 5: the S-C node kernel with the claimer union + join masks -- PARTIAL parity, then an A/B of the
# S-C bench against the previous commit's library (var_ab/libgm_base.so), twice each, and the SQ mix
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05g}
mkdir -p $O
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PT tests/test_gpu_partial.py tests/test_gpu_msgcount.py -m gpu -k "partial or row_shard or packed or half or msgcount" \
  > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -3 $O/gpu_tests.txt
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
for k in 1 2; do
  timeout -k 10 300 python3 bench.py --scenario S-C --no-cpu --no-pmc --steps 10 --warmup 2 > $O/sc_new_$k.json 2> $O/sc_new_$k.err || exit 1
  GM_AB_BUILD=1 GM_LIBRARY=var_ab/libgm_base.so timeout -k 10 300 python3 bench.py --scenario S-C --no-cpu --no-pmc --steps 10 --warmup 2 > $O/sc_base_$k.json 2> $O/sc_base_$k.err || exit 1
done
bash scripts/gpu.sh ${1:-r05g} mix_sc
rc=$?
for f in $O/sc_*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f', d['roofline']['kernel_ms'], d['ms_per_step'])"; done
exit $rc
