#!/bin/bash
# round-4: S-C small kernel reads the union through its list of claimed slots (no sweep of all
# 512 table slots, no compaction pass) -- PARTIAL parity, then the S-C bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04zd
mkdir -p $O
TESTS="tests/test_gpu_partial.py tests/test_gpu_msgcount.py tests/test_gpu_baseline_configs.py tests/test_gpu_fullsize_shards.py" \
  bash scripts/gpu.sh r04zd tests || exit 1
BENCH_ARGS="--no-cpu" bash scripts/gpu.sh r04zd sc
