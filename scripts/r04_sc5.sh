#!/bin/bash
# round-4: S-C draw's Lemire threshold from a constant table (no 32-bit remainder per node) --
# PARTIAL parity, then an A/B against the previous gm_partial.hip (varlib/scprev) on this box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TESTS="tests/test_gpu_partial.py tests/test_gpu_msgcount.py tests/test_gpu_baseline_configs.py" \
  bash scripts/gpu.sh r04zo tests || exit 1
AB_TAG=r04zo bash scripts/r04_sc_ab.sh
