#!/bin/bash
# round-4: the entry pass and fast_cell branch-free (selects, unconditional LDS or / add) -- parity,
# per-tick times and SQ mix
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04zb
mkdir -p $O
TESTS="tests/test_gpu_band_fast.py tests/test_gpu_scaled.py tests/test_gpu_baseline_configs.py tests/test_gpu_msgcount.py tests/test_gpu_sharded.py tests/test_gpu_limits.py tests/test_gpu_ramp.py" \
  bash scripts/gpu.sh r04zb tests || exit 1
timeout -k 10 200 python -u scripts/tick_times.py 65536 48 > $O/tick_times.txt 2>&1 || exit 1
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/mix_fast -o p -- \
  python3 scripts/tick_times.py 65536 48 > $O/mix_fast.log 2>&1 || exit 1
python3 scripts/pmc_per_dispatch.py gm_s_band_fast $O/mix_fast/p_counter_collection.csv > $O/mix_fast.txt
