#!/bin/bash
# round 5, first GPU call: shard breakdown profiles + the tests the first commits touch
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05b}
mkdir -p $O
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PT tests/test_gpu_partial.py tests/test_gpu_faithful.py tests/test_gpu_limits.py \
  tests/test_gpu_baseline_configs.py -m gpu --durations 10 > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -3 $O/gpu_tests.txt
bash scripts/r05/prof_shard.sh ${1:-r05b}
