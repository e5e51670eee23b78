#!/bin/bash
# SCALED join ramp parity vs the oracle (+ the existing SCALED suite as a regression check).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/w
timeout -k 10 600 python -u -m pytest tests/test_gpu_ramp.py -x -v --timeout 300 --timeout-method thread > gpurun_out/w/t_ramp.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_scaled.py -x -q --timeout 300 --timeout-method thread > gpurun_out/w/t_scaled.log 2>&1
rc=$?
echo "rc=$rc"; grep -E "PASS|FAIL|passed|failed|Error|assert" gpurun_out/w/t_ramp.log | tail -12; tail -n 2 gpurun_out/w/t_scaled.log
exit $rc
