#!/bin/bash
# A/B of the TREMOVE-tick removal scatter (gm_s_band_fast quick path): band-fast + SCALED parity tests,
# then per-tick band times of the S-A schedule, new tree vs the previous library (OLD_LIB, default build_dbg/head),
# interleaved twice on one box.
# usage: scripts/r06/ab_gone.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_band_fast.py tests/test_gpu_scaled.py tests/test_gpu_baseline_configs.py > $O/gpu_tests.txt 2>&1 || { tail -5 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
for i in 1 2; do
  timeout -k 10 200 python3 -u scripts/tick_times.py 65536 > $O/ticks_new_$i.txt 2>&1 || exit 1
  GM_AB_BUILD=1 GM_LIBRARY=${OLD_LIB:-build_dbg/head/libgm.so} timeout -k 10 200 python3 -u scripts/tick_times.py 65536 > $O/ticks_old_$i.txt 2>&1 || exit 1
done
for f in $O/ticks_*.txt; do echo "$f $(awk '$2>=29 && $2<=48 {s+=$4; n++} END {printf "window %.3f ms/tick (%d ticks)", s/n, n}' $f)"; done
