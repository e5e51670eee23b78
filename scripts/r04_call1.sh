#!/bin/bash
# round-4 GPU call: S-C ablation builds (scripts/sc_variants.sh), then the new/affected GPU tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
VARIANTS="main defer nodrop prof nowait" bash scripts/sc_ablate.sh || exit 1
TESTS="tests/test_gpu_gloo_shards.py tests/test_gpu_fullsize_shards.py tests/test_gpu_limits.py tests/test_gpu_baseline_configs.py tests/test_gpu_sharded.py tests/test_gpu_partial.py tests/test_gpu_scaled.py" bash scripts/gpu.sh r04b tests
