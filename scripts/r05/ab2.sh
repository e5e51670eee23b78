#!/bin/bash
# round 5: A/B of S-C node-kernel variants (var_ab/*.so, interleaved, two runs each) and the S-A
# four-rows-per-wave draw (gm_s_pick0 vs GM_PICK0=0), after the SCALED / PARTIAL parity tests of the tree's library
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05h}
mkdir -p $O
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PT tests/test_gpu_scaled.py tests/test_gpu_band_fast.py tests/test_gpu_ramp.py tests/test_gpu_partial.py \
  tests/test_gpu_baseline_configs.py -m gpu > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -3 $O/gpu_tests.txt
for k in 1 2; do
  for v in base sweep_jm claim1 claim2; do
    GM_AB_BUILD=1 GM_LIBRARY=var_ab/libgm_$v.so timeout -k 10 300 python3 bench.py --scenario S-C --no-cpu --no-pmc --steps 10 --warmup 2 \
      > $O/sc_${v}_$k.json 2> $O/sc_${v}_$k.err || exit 1
  done
  timeout -k 10 300 python3 bench.py --no-cpu --no-pmc --no-companion > $O/sa_pick0_$k.json 2> $O/sa_pick0_$k.err || exit 1
  GM_PICK0=0 timeout -k 10 300 python3 bench.py --no-cpu --no-pmc --no-companion > $O/sa_pick_$k.json 2> $O/sa_pick_$k.err || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sa -o sa -- python3 bench.py --no-cpu --no-pmc --no-companion > $O/prof_sa.log 2>&1
for f in $O/sc_*.json $O/sa_*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f', round(d['roofline']['kernel_ms'],3), round(d['ms_per_step'],3), round(d['value']/1e6,2))"; done
