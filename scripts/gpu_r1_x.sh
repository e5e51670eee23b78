#!/bin/bash
# Join ramp at scale (N = 16,384, the whole 4,096-tick ramp) on the GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/x
timeout -k 10 600 python -u -m pytest tests/test_gpu_ramp.py -x -v --timeout 500 --timeout-method thread -k scale --durations=3 > gpurun_out/x/t.log 2>&1
rc=$?
echo "rc=$rc"; grep -E "PASS|FAIL|passed|failed|Error|assert|call" gpurun_out/x/t.log | tail -12
exit $rc
