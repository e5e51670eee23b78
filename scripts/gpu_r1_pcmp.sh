#!/bin/bash
# PARTIAL kernel variants side by side (GM_LIBRARY per variant): per-wave instruction mix
# (one PMC pass each, kernel trace for durations) at S-C N = 4M, plus S-C HBM traffic passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/pcmp
mkdir -p $O
B="python3 bench.py --scenario S-C --cluster 4194304 --no-cpu --steps 4 --warmup 1 --prologue 12"
rc=0
for v in ${VARIANTS:-base v2}; do
  GM_LIBRARY=distributed-membership_amd/lib/libgm_$v.so timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES --kernel-trace --output-format csv -d $O/$v -o p1 -- $B > $O/$v.log 2>&1 || { rc=$?; break; }
done
if [ $rc -eq 0 ] && [ -n "$TRAFFIC" ]; then
  B2="python3 bench.py --scenario S-C --no-cpu --steps 3 --warmup 1"
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o f -- $B2 > $O/fetch.log 2>&1 &&
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write -o w -- $B2 > $O/write.log 2>&1
  rc=$?
fi
echo "rc=$rc"
exit $rc
