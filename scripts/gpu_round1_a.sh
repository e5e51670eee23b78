#!/bin/bash
# First GPU pass: faithful parity subset, scaled parity subset, a short bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest tests/test_gpu_faithful.py -x -q --timeout 120 --timeout-method thread \
  -k "singlefailure_T42_R7 or multifailure_T1_R1 or msgdropsinglefailure_T42_R7" > gpurun_out/t_faith.log 2>&1 &&
timeout -k 10 240 python -u -m pytest tests/test_gpu_scaled.py -x -q --timeout 120 --timeout-method thread \
  -k "64 or 128" > gpurun_out/t_scaled.log 2>&1 &&
timeout -k 10 200 python -u bench.py --cluster 16384 --steps 10 --warmup 2 --no-cpu > gpurun_out/b16k.log 2>&1
rc=$?
echo "rc=$rc"
tail -5 gpurun_out/t_faith.log gpurun_out/t_scaled.log gpurun_out/b16k.log 2>/dev/null
exit $rc
