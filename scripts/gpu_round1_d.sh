#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sharded.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_shard.log 2>&1
rc=$?
echo "rc=$rc"; tail -n 30 gpurun_out/t_shard.log
exit $rc
