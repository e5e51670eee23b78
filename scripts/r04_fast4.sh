#!/bin/bash
# round-4: the fast path's evcum cell read with the metadata and written back plainly (no atomic),
# 16,384 event-total stripes -- parity, then per-tick times
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04p
mkdir -p $O
TESTS="tests/test_gpu_band_fast.py tests/test_gpu_scaled.py tests/test_gpu_baseline_configs.py tests/test_gpu_msgcount.py tests/test_gpu_sharded.py tests/test_gpu_limits.py" \
  bash scripts/gpu.sh r04p tests || exit 1
timeout -k 10 200 python -u scripts/tick_times.py 65536 48 > $O/tick_times.txt 2>&1 || exit 1
BENCH_ARGS="--no-cpu --no-pmc --no-companion" bash scripts/gpu.sh r04p sa
