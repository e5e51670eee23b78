#!/bin/bash
# round 5 closing gate, part A: the whole GPU suite, smoke, the default bench (S-A with the S-B
# companion, live PMC traffic and the CPU baseline), S-C -- with the last segment of the hour-sized
# CPU run (scripts/cpu_hour.py, N = 13,722, one host core) in the background for the call's length.
#   usage: scripts/r05/gate_final_a.sh <tag> <cpu segment start tick>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-r05o}
O=gpurun_out/$TAG
mkdir -p $O
CPU_PID=
if [ -n "$2" ]; then
  timeout -k 10 1100 python3 -u scripts/cpu_hour.py --cluster 13722 --start $2 --ticks 25 \
    --out $O/cpu_hour_seg$2.jsonl > $O/cpu_hour_seg$2.log 2>&1 &
  CPU_PID=$!
fi
bash scripts/gpu.sh $TAG tests smoke sa sc
rc=$?
tail -3 $O/gpu_tests.txt
[ $rc -ne 0 ] && { echo "gate failed"; [ -n "$CPU_PID" ] && kill $CPU_PID; exit 1; }
for f in $O/bench_sa.json $O/bench_sc.json; do cut -c1-600 $f; done
if [ -n "$CPU_PID" ]; then wait $CPU_PID; echo "cpu segment rc=$?"; tail -2 $O/cpu_hour_seg$2.jsonl; fi
exit $rc
