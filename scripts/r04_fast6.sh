#!/bin/bash
# round-4: where the escape-window ticks spend their time -- per-tick SQ mix of the fast kernel, and
# per-tick times with every unit forced through the per-cell pass (varlib/always)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04w
mkdir -p $O
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/mix_fast -o p -- \
  python3 scripts/tick_times.py 65536 48 > $O/mix_fast.log 2>&1 || exit 1
python3 scripts/pmc_per_dispatch.py gm_s_band_fast $O/mix_fast/p_counter_collection.csv > $O/mix_fast.txt
GM_AB_BUILD=1 GM_LIBRARY=varlib/always/libgm.so timeout -k 10 200 python -u scripts/tick_times.py 65536 48 > $O/tick_times_always.txt 2>&1 || exit 1
timeout -k 10 200 python -u scripts/tick_times.py 65536 48 > $O/tick_times_main.txt 2>&1 || exit 1
