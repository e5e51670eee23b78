#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
VARIANTS="main route" bash scripts/sc_ablate.sh || exit 1
GM_AB_BUILD=1 GM_LIBRARY=build_var/route/libgm.so timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_partial.py > gpurun_out/abl/route_partial_tests.txt 2>&1
echo "route partial tests rc=$?" >> gpurun_out/abl/steps.txt
TESTS="tests/test_gpu_fullsize_shards.py tests/test_gpu_limits.py tests/test_gpu_baseline_configs.py" bash scripts/gpu.sh r04c tests
