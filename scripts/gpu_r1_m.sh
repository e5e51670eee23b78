#!/bin/bash
# PARTIAL-view parity on the GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_partial.py -x -v --timeout 200 --timeout-method thread > gpurun_out/t_partial.log 2>&1
rc=$?
echo "rc=$rc"; grep -E "PASS|FAIL|Error|assert|differ" gpurun_out/t_partial.log | head -20
exit $rc
