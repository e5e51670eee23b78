#!/bin/bash
# PMC traffic passes (separate runs per counter group, kernel-trace only), then
# a second plain bench run to gauge run-to-run variance.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
N=${N:-65536}
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch -o r01 -- python3 bench.py --no-cpu --cluster $N --steps 5 --warmup 1 > gpurun_out/pmc_fetch.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write -o r01 -- python3 bench.py --no-cpu --cluster $N --steps 5 --warmup 1 > gpurun_out/pmc_write.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/bench2.log 2>&1
rc=$?
echo "rc=$rc"
ls gpurun_out/pmc_fetch gpurun_out/pmc_write; cat gpurun_out/bench2.log
exit $rc
