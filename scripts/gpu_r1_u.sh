#!/bin/bash
# PARTIAL kernel iteration: parity (fast subset), S-C bench, PMC instruction mix.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/it
timeout -k 10 400 python -u -m pytest tests/test_gpu_partial.py -x -q --timeout 300 --timeout-method thread > gpurun_out/it/t.log 2>&1 &&
timeout -k 10 300 python -u bench.py --scenario S-C --no-cpu > gpurun_out/it/bench.log 2>&1 &&
bash scripts/gpu_r1_p.sh > gpurun_out/it/pmc.log 2>&1
rc=$?
echo "rc=$rc"; tail -n 2 gpurun_out/it/t.log; tail -n 1 gpurun_out/it/bench.log | cut -c1-400; grep -E "SQ_" gpurun_out/it/pmc.log
exit $rc
