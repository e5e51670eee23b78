#!/bin/bash
# round-4: S-C small kernel with the view width folded in (V = 32 instantiation) and a full-rate
# table hash -- PARTIAL parity, then the S-C bench (tick kernels by HIP events)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04zc
mkdir -p $O
TESTS="tests/test_gpu_partial.py tests/test_gpu_msgcount.py tests/test_gpu_baseline_configs.py tests/test_gpu_fullsize_shards.py" \
  bash scripts/gpu.sh r04zc tests || exit 1
BENCH_ARGS="--no-cpu" bash scripts/gpu.sh r04zc sc
