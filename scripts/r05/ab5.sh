#!/bin/bash
# round 5: (1) S-A, three interleaved rounds of the bench and two of the per-tick times: the tree (two
# bands per wave, hook 3, KP) against var_fast/ head (the last commit's kernel), b2h0 and b1;
# (2) S-B: the stub shard and the G = 8 pipelined loopback at K = 2 vs 4 exchange chunks;
# (3) one CPU-hour segment in the background.   usage: ab5.sh <tag> <cpu start>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05m}
mkdir -p $O
CPU_PID=
if [ -n "$2" ]; then
  timeout -k 10 1000 python3 -u scripts/cpu_hour.py --cluster 13722 --start $2 --ticks 25 \
    --out $O/cpu_hour_seg$2.jsonl > $O/cpu_hour_seg$2.log 2>&1 &
  CPU_PID=$!
fi
fail() { echo "$1"; [ -n "$CPU_PID" ] && kill $CPU_PID; exit 1; }
for k in 1 2 3; do
  timeout -k 10 300 python3 bench.py --no-cpu --no-pmc --no-companion > $O/sa_tree_$k.json 2> $O/sa_tree_$k.err || fail "bench tree"
  for v in head b2h0 b1; do
    GM_AB_BUILD=1 GM_LIBRARY=var_fast/libgm_$v.so timeout -k 10 300 python3 bench.py --no-cpu --no-pmc --no-companion > $O/sa_${v}_$k.json 2> $O/sa_${v}_$k.err || fail "bench $v"
  done
done
for f in $O/sa_*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f', round(d['roofline']['kernel_ms'],3), round(d['ms_per_step'],3), round(d['value']/1e6,2))"; done
for k in 1 2; do
  timeout -k 10 300 python -u scripts/tick_times.py 65536 > $O/ticks_tree_$k.txt 2>&1 || fail "ticks"
  GM_AB_BUILD=1 GM_LIBRARY=var_fast/libgm_head.so timeout -k 10 300 python -u scripts/tick_times.py 65536 > $O/ticks_head_$k.txt 2>&1 || fail "ticks head"
done
for f in $O/ticks_*.txt; do python3 -c "
import re,sys
v={int(m.group(1)):float(m.group(2)) for m in re.finditer(r't=\s*(\d+) band\s+([\d.]+)', open('$f').read())}
st=[v[t] for t in range(14,23)]; es=[v[t] for t in range(23,31)]; w=[v[t] for t in range(29,49)]
print('$f', 'steady', round(sum(st)/len(st),3), 'escape', round(sum(es)/len(es),3), 'window', round(sum(w)/len(w),3))"; done
for K in 2 4; do
  GM_SCHUNKS=$K timeout -k 10 300 python3 scripts/shard_profile.py --sb > $O/sb_stub_k$K.json 2> $O/sb_stub_k$K.err || fail "sb stub $K"
  GM_SCHUNKS=$K timeout -k 10 600 python3 scripts/sb_loopback_profile.py --pipelined > $O/sb_loop_k$K.json 2> $O/sb_loop_k$K.err || fail "sb loop $K"
done
for f in $O/sb_stub_k*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f', round(d['ms_per_tick'],3), round(d['band_kernel_ms'],3))"; done
for f in $O/sb_loop_k*.json; do cut -c1-400 $f; done
if [ -n "$CPU_PID" ]; then wait $CPU_PID; echo "cpu segment rc=$?"; tail -2 $O/cpu_hour_seg$2.jsonl; fi
