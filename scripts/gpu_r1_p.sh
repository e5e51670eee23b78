#!/bin/bash
# S-C gm_p_tick PMC: instruction mix and stall split (one counter group per pass).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/scpmc
B="python3 bench.py --scenario S-C --cluster 4194304 --no-cpu --steps 4 --warmup 1 --prologue 12"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --kernel-trace --output-format csv -d gpurun_out/scpmc/p1 -o p1 -- $B > gpurun_out/scpmc/p1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/scpmc/p2 -o p2 -- $B > gpurun_out/scpmc/p2.log 2>&1
rc=$?
echo "rc=$rc"
for f in $(find gpurun_out/scpmc -name '*counter_collection.csv'); do python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(float); cnt = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    if "gm_p_tick_small" not in r.get("Kernel_Name", ""): continue
    acc[r["Counter_Name"]] += float(r["Counter_Value"]); cnt[r["Counter_Name"]] += 1
for k in sorted(acc): print(k, acc[k] / max(1, cnt[k]) * 1.0, "(per-dispatch avg over", cnt[k], "rows)")
PY
done
exit $rc
