#!/bin/bash
# G=8 column-shard loopback parity + PARTIAL parity + S-C bench after the removal fast path.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/aa
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_partial.py -x -q --timeout 300 --timeout-method thread -k "2048-8 or partial or row_shards" > gpurun_out/aa/t.log 2>&1 &&
timeout -k 10 300 python -u bench.py --scenario S-C --no-cpu > gpurun_out/aa/bench_sc.log 2>&1
rc=$?
echo "rc=$rc"; tail -n 3 gpurun_out/aa/t.log; tail -n 1 gpurun_out/aa/bench_sc.log | cut -c1-220
exit $rc
