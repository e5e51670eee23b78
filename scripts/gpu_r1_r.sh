#!/bin/bash
# RCCL rehearsal on one GPU: sharded tests (loopback + single-rank RCCL), then the
# forced-shard bench (the multi-GPU tick protocol at G=1) next to the fused bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/rccl
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py -x -v --timeout 300 --timeout-method thread > gpurun_out/rccl/t_sharded.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu --force-shard > gpurun_out/rccl/bench_force_shard.log 2>&1
rc=$?
echo "rc=$rc"; grep -E "passed|failed|Error|assert" gpurun_out/rccl/t_sharded.log | tail -5; tail -n 3 gpurun_out/rccl/bench_force_shard.log
exit $rc
