#!/bin/bash
# PARTIAL kernel iteration: S-C parity tests, S-C bench, kernel trace of the S-C bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
D=gpurun_out/${PC_TAG:-pc}
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_partial.py -x -q --timeout 300 --timeout-method thread > $D/tests.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --scenario S-C --no-cpu > $D/bench_sc.json 2> $D/bench_sc.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o sc -- python3 bench.py --scenario S-C --no-cpu --steps 10 > $D/prof.log 2>&1
rc=$?
echo "rc=$rc"; tail -n 2 $D/tests.txt; cat $D/bench_sc.json
exit $rc
