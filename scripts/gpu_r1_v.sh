#!/bin/bash
# Chunk-pipelined row shards (parity) + FAITHFUL at N=1000 (max EmulNet size) + S-C bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/v
timeout -k 10 600 python -u -m pytest tests/test_gpu_partial.py -x -v --timeout 300 --timeout-method thread > gpurun_out/v/t_partial.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_faithful.py -x -v --timeout 300 --timeout-method thread -k "n1000 or n520" > gpurun_out/v/t_faithful.log 2>&1 &&
timeout -k 10 300 python -u bench.py --scenario S-C --no-cpu --force-shard > gpurun_out/v/bench_force.log 2>&1
rc=$?
echo "rc=$rc"; grep -E "PASS|FAIL|passed|failed|Error" gpurun_out/v/t_partial.log | tail -14; grep -E "PASS|FAIL|passed|failed|Error" gpurun_out/v/t_faithful.log | tail -3; tail -n 1 gpurun_out/v/bench_force.log | cut -c1-250
exit $rc
