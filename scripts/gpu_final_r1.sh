#!/bin/bash
# Round gate: full GPU parity suite, smoke, S-A bench (with cpu baseline), S-C bench
# (with cpu baseline), rocprofv3 kernel-trace --stats of both benches (CSV).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations 12 > $O/gpu_tests.txt 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 &&
timeout -k 10 240 python -u bench.py > $O/bench_sa.json 2> $O/bench_sa.err &&
timeout -k 10 300 python -u bench.py --scenario S-C > $O/bench_sc.json 2> $O/bench_sc.err &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sa -o sa -- python3 bench.py --no-cpu > $O/prof_sa.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sc -o sc -- python3 bench.py --scenario S-C --no-cpu > $O/prof_sc.log 2>&1
rc=$?
echo "rc=$rc"; tail -n 3 $O/gpu_tests.txt; tail -n 1 $O/smoke.txt; cut -c1-300 $O/bench_sa.json; cut -c1-300 $O/bench_sc.json
exit $rc
