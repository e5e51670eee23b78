#!/bin/bash
# round 5: gm_s_pick0 with the band records chunk counts in LDS (one load per draw, not two)
# -- SCALED / band-fast / shard parity on the tree, then three interleaved
# rounds of the S-A bench and two of the per-tick times, tree against var_q/libgm_nomul.so (the last commit).
#   usage: ab8.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05x}
mkdir -p $O
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PT tests/test_gpu_band_fast.py tests/test_gpu_scaled.py tests/test_gpu_sharded.py tests/test_gpu_limits.py -m gpu > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
for k in 1 2 3; do
  timeout -k 10 300 python3 bench.py --no-cpu --no-pmc --no-companion > $O/sa_tree_$k.json 2> $O/sa_tree_$k.err || exit 1
  GM_AB_BUILD=1 GM_LIBRARY=var_q/libgm_nomul.so timeout -k 10 300 python3 bench.py --no-cpu --no-pmc --no-companion > $O/sa_base_$k.json 2> $O/sa_base_$k.err || exit 1
done
for f in $O/sa_*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f', round(d['roofline']['kernel_ms'],3), round(d['ms_per_step'],3), round(d['value']/1e6,2))"; done
for k in 1 2; do
  timeout -k 10 300 python -u scripts/tick_times.py 65536 > $O/ticks_tree_$k.txt 2>&1 || exit 1
  GM_AB_BUILD=1 GM_LIBRARY=var_q/libgm_nomul.so timeout -k 10 300 python -u scripts/tick_times.py 65536 > $O/ticks_base_$k.txt 2>&1 || exit 1
done
for f in $O/ticks_*.txt; do python3 -c "
import re
v={int(m.group(1)):float(m.group(2)) for m in re.finditer(r't=\s*(\d+) band\s+([\d.]+)', open('$f').read())}
g=lambda a,b: round(sum(v[t] for t in range(a,b))/(b-a),3)
print('$f', 'steady', g(14,23), 'esc23-30', g(23,31), 'trem31-38', g(31,39), 'window', g(29,49))"; done
