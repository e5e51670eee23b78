#!/bin/bash
# round 5 full gate: GPU test suite, smoke, the default bench (S-A + S-B companion, live PMC, CPU
# baseline), S-C, the S-B stub shard and G = 8 loopback, the S-A rocprof stats -- with one segment
# of the hour-sized CPU baseline run (scripts/cpu_hour.py, N = 13,722, one host core) in the
# background on the box's CPU for the call's length.
#   usage: scripts/r05/gate_full.sh <tag> <cpu segment start tick> <ticks>   (start 0: from the warm start)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-r05f}
O=gpurun_out/$TAG
mkdir -p $O
CPU_PID=
if [ -n "$2" ]; then
  timeout -k 10 ${CPU_LIMIT:-1100} python3 -u scripts/cpu_hour.py --cluster 13722 --start $2 --ticks ${3:-25} \
    --out $O/cpu_hour_seg$2.jsonl > $O/cpu_hour_seg$2.log 2>&1 &
  CPU_PID=$!
fi
bash scripts/gpu.sh $TAG tests smoke sa sc || { echo "gate failed"; [ -n "$CPU_PID" ] && kill $CPU_PID; exit 1; }
timeout -k 10 300 python3 scripts/shard_profile.py --sb > $O/sb_stub.json 2> $O/sb_stub.err &&
timeout -k 10 300 python3 scripts/shard_profile.py --sb --cluster 65536 > $O/sa_stub.json 2> $O/sa_stub.err &&
timeout -k 10 600 python3 scripts/sb_loopback_profile.py --pipelined > $O/sb_loopback_pipe.json 2> $O/sb_loopback_pipe.err &&
bash scripts/gpu.sh $TAG prof_sa ticks
rc=$?
# bisect of the S-A band-kernel time over round-5 commits (var_ab/libgm_<commit>.so), when present
if [ $rc -eq 0 ] && ls var_ab/libgm_*.so > /dev/null 2>&1; then
  for L in var_ab/libgm_*.so; do
    v=$(basename $L .so)
    GM_AB_BUILD=1 GM_LIBRARY=$L timeout -k 10 300 python3 bench.py --no-cpu --no-pmc --no-companion > $O/bisect_$v.json 2> $O/bisect_$v.err || break
    python3 -c "import json;d=json.load(open('$O/bisect_$v.json'));print('$v', round(d['roofline']['kernel_ms'],3), round(d['ms_per_step'],3))"
  done
fi
if [ -n "$CPU_PID" ]; then wait $CPU_PID; echo "cpu segment rc=$?"; tail -2 $O/cpu_hour_seg$2.jsonl; fi
for f in $O/sb_stub.json $O/sa_stub.json $O/sb_loopback_pipe.json; do [ -f $f ] && cut -c1-300 $f; done
exit $rc
