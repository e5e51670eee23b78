#!/bin/bash
# round-4: fast path per-tick instruction mix (SQ counters per launch) against the general path
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04k
mkdir -p $O
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
timeout -k 10 200 python -u scripts/tick_times.py 65536 48 > $O/tick_times.txt 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/mix_fast -o p -- \
  python3 scripts/tick_times.py 65536 48 > $O/mix_fast.log 2>&1 || exit 1
GM_BAND_FAST=0 timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/mix_gen -o p -- \
  python3 scripts/tick_times.py 65536 48 > $O/mix_gen.log 2>&1 || exit 1
python3 scripts/pmc_per_dispatch.py gm_s_band_fast $O/mix_fast/p_counter_collection.csv > $O/mix_fast.txt
python3 scripts/pmc_per_dispatch.py "gm_s_band<" $O/mix_gen/p_counter_collection.csv > $O/mix_gen.txt
