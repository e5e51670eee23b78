#!/bin/bash
# Full GPU gate: parity suite and smoke (RCCL needs distinct devices: multi-rank runs only on the 8-GPU node).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?
echo "rc=$rc"; tail -n 3 gpurun_out/t_all.log; tail -n 2 gpurun_out/smoke.log; tail -n 3 gpurun_out/two_rank.log
exit $rc
