#!/bin/bash
# sharded path: parity (loopback) + kernel profile of 8 shards of N=65536 on one device.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_scaled.py tests/test_gpu_sharded.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_scaled.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/psh -o r --output-format csv -- python3 scripts/shard_profile.py > gpurun_out/psh.log 2>&1
rc=$?
echo "rc=$rc"; tail -n 2 gpurun_out/t_scaled.log; grep "ms/tick" gpurun_out/psh.log; cat gpurun_out/psh/r_kernel_stats.csv
exit $rc
