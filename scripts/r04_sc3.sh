#!/bin/bash
# round-4: S-C table sweep with one compare per slot for the alive bit (removals = present - alive)
# -- PARTIAL parity, then an A/B against the previous gm_partial.hip (varlib/scprev) on this box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TESTS="tests/test_gpu_partial.py tests/test_gpu_msgcount.py tests/test_gpu_baseline_configs.py tests/test_gpu_fullsize_shards.py" \
  bash scripts/gpu.sh r04zf tests || exit 1
AB_TAG=r04zf bash scripts/r04_sc_ab.sh
