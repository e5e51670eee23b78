#!/bin/bash
# round-4: escaped cells of the fast path entry-parallel (lane j takes escape entry j) -- parity,
# then per-tick times and the S-A bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04v
mkdir -p $O
TESTS="tests/test_gpu_band_fast.py tests/test_gpu_scaled.py tests/test_gpu_baseline_configs.py tests/test_gpu_msgcount.py tests/test_gpu_sharded.py tests/test_gpu_limits.py tests/test_gpu_fullsize_shards.py tests/test_gpu_ramp.py" \
  bash scripts/gpu.sh r04v tests || exit 1
timeout -k 10 200 python -u scripts/tick_times.py 65536 48 > $O/tick_times.txt 2>&1 || exit 1
BENCH_ARGS="--no-cpu --no-pmc --no-companion" bash scripts/gpu.sh r04v sa
