#!/bin/bash
# round-4: S-C small kernel at 16 nodes per wave -- PARTIAL parity, then an A/B against 32 nodes
# per wave (varlib/npw32) on this box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TESTS="tests/test_gpu_partial.py tests/test_gpu_msgcount.py tests/test_gpu_baseline_configs.py tests/test_gpu_fullsize_shards.py" \
  bash scripts/gpu.sh r04zk tests || exit 1
AB_TAG=r04zk VARS="npw32" bash scripts/r04_sc_ab.sh
