#!/bin/bash
# round-4: striped packed row-shard records + S-C kernel variants (wire lists, packed table, staged lists)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04e
mkdir -p $O
TESTS="tests/test_gpu_partial.py tests/test_gpu_fullsize_shards.py" bash scripts/gpu.sh r04e tests || exit 1
timeout -k 10 300 python -u scripts/partial_shard_profile.py > $O/pshard_g8.json 2> $O/pshard_g8.err || exit 1
timeout -k 10 300 python -u bench.py --scenario S-C --no-cpu > $O/bench_sc.json 2> $O/bench_sc.err || exit 1
vt() {  # parity of a variant library: the PARTIAL tests
  GM_AB_BUILD=1 GM_LIBRARY=build_var/$1/libgm.so timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread \
    tests/test_gpu_partial.py "tests/test_gpu_fullsize_shards.py::test_sc_full_size_row_shards_match_single_context" \
    tests/test_gpu_msgcount.py tests/test_gpu_baseline_configs.py -k "partial or sc_ or events" > $O/$1_tests.txt 2>&1
  local rc=$?
  echo "$1 tests rc=$rc" >> $O/steps.txt
  case $rc in 124|134|137|139) exit 1 ;; esac  # a hang or a fault: no further GPU step
  return $rc
}
vt staged || vt packed || vt wire
VARIANTS="main wire packed staged" bash scripts/sc_ablate.sh
