#!/bin/bash
# round-4: gm_s_band fast path (byte-domain merge + SWAR sweep, per-cell fixups) -- the full GPU
# suite (the byte range rule changed for every path), then timing
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TESTS="tests/test_gpu_band_fast.py tests/test_gpu_scaled.py tests" bash scripts/gpu.sh r04j tests || exit 1
BENCH_ARGS="--no-cpu --no-pmc --no-companion" bash scripts/gpu.sh r04j sa ticks prof_sa
