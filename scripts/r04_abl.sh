#!/bin/bash
# round-4 ablation: TREMOVE ticks without the event atomics / without atomics and records (measurement builds)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r04o
mkdir -p $O
timeout -k 10 200 python -u scripts/tick_times.py 65536 48 > $O/tick_times_main.txt 2>&1 || exit 1
GM_LIBRARY=varlib/noatom/libgm.so timeout -k 10 200 python -u scripts/tick_times.py 65536 48 > $O/tick_times_noatom.txt 2>&1 || exit 1
GM_LIBRARY=varlib/both/libgm.so timeout -k 10 200 python -u scripts/tick_times.py 65536 48 > $O/tick_times_both.txt 2>&1 || exit 1
