#!/bin/bash
# PARTIAL row shards: parity (loopback exchange) + single-GPU S-C bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/sc3
timeout -k 10 600 python -u -m pytest tests/test_gpu_partial.py -x -v --timeout 400 --timeout-method thread > gpurun_out/sc3/t_partial.log 2>&1 &&
timeout -k 10 300 python -u bench.py --scenario S-C --no-cpu > gpurun_out/sc3/bench.log 2>&1
rc=$?
echo "rc=$rc"; grep -E "PASS|FAIL|passed|failed|Error|assert" gpurun_out/sc3/t_partial.log | tail -12; tail -n 1 gpurun_out/sc3/bench.log
exit $rc
