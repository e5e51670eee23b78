#!/bin/bash
# Re-entry check after a container rebuild: full GPU parity suite, smoke, default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench_n.log 2>&1
rc=$?
echo "rc=$rc"; tail -n 3 gpurun_out/t_all.log; tail -n 2 gpurun_out/smoke.log; tail -n 1 gpurun_out/bench_n.log
exit $rc
