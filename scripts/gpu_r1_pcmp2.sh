#!/bin/bash
# PARTIAL variants: parity tests on the default libgm (the newest variant), then per variant
# (GM_LIBRARY) an S-C N=16M bench and a per-wave instruction-mix PMC pass at N = 4M.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-pcmp2}
mkdir -p $O
B="python3 bench.py --scenario S-C --cluster 4194304 --no-cpu --steps 4 --warmup 1 --prologue 12"
timeout -k 10 400 python -u -m pytest tests/test_gpu_partial.py -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
rc=$?
for v in ${VARIANTS:-base v3 v4}; do
  [ $rc -eq 0 ] || break
  GM_LIBRARY=distributed-membership_amd/lib/libgm_$v.so timeout -k 10 200 python3 -u bench.py --scenario S-C --no-cpu > $O/bench_$v.json 2> $O/bench_$v.err || { rc=$?; break; }
  GM_LIBRARY=distributed-membership_amd/lib/libgm_$v.so timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES --kernel-trace --output-format csv -d $O/$v -o p1 -- $B > $O/$v.log 2>&1 || { rc=$?; break; }
done
echo "rc=$rc"; tail -n 2 $O/tests.txt
for v in ${VARIANTS:-base v3 v4}; do python3 -c "import json,sys; d=json.load(open('$O/bench_$v.json')); print('$v', d['ms_per_step'], d['roofline']['kernel_ms'])" 2>/dev/null; done
exit $rc
