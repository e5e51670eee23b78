#!/bin/bash
# round-4 experiment: gm_s_band_fast with two bands per wave (measurement build varlib/fb2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r04n
mkdir -p $O
timeout -k 10 200 python -u scripts/tick_times.py 65536 48 > $O/tick_times_main.txt 2>&1 || exit 1
GM_LIBRARY=varlib/fb2/libgm.so timeout -k 10 200 python -u scripts/tick_times.py 65536 48 > $O/tick_times_fb2.txt 2>&1 || exit 1
GM_LIBRARY=varlib/fb2/libgm.so timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread \
  tests/test_gpu_band_fast.py -m gpu > $O/fb2_tests.txt 2>&1
