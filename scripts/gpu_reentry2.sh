#!/bin/bash
# Re-entry gate: full GPU parity suite, smoke, default S-A bench (with cpu baseline).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/re2
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/re2/gpu_tests.txt 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/re2/smoke.txt 2>&1 &&
timeout -k 10 240 python -u bench.py > gpurun_out/re2/bench_sa.json 2> gpurun_out/re2/bench_sa.err
rc=$?
echo "rc=$rc"; tail -n 3 gpurun_out/re2/gpu_tests.txt; tail -n 2 gpurun_out/re2/smoke.txt; cat gpurun_out/re2/bench_sa.json
exit $rc
