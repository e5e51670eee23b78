#!/bin/bash
# A/B of an S-C tick-kernel change: the PARTIAL parity tests, then bench.py --scenario S-C with the new
# tree and with the previous library (OLD_LIB, default build_dbg/head), interleaved three times.
# usage: scripts/r06/ab_sc.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_partial.py tests/test_gpu_msgcount.py tests/test_gpu_limits.py > $O/gpu_tests.txt 2>&1 || { tail -5 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
B="python3 bench.py --scenario S-C --no-cpu --no-pmc --steps 10 --warmup 2"
for i in 1 2 3; do
  timeout -k 10 200 $B > $O/new_$i.json 2>/dev/null || exit 1
  GM_AB_BUILD=1 GM_LIBRARY=${OLD_LIB:-build_dbg/head/libgm.so} timeout -k 10 200 $B > $O/old_$i.json 2>/dev/null || exit 1
done
for f in $O/new_*.json $O/old_*.json; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3))"; done
