#!/bin/bash
# round 5: the fast band kernel at two bands per wave (the second unit's table slice and gathers issued
# under the first unit's stores) and the row's kernel-argument words in one batch (GM_KP) --
# correctness on the tree build, then S-A band-kernel time of the tree (2 bands, hook 3, KP) against
# var_fast/ builds, interleaved: b1 (1 band, KP), b1kp0 (1 band, no KP), b2h0 (2 bands, second unit's
# loads after the first unit), h1 (loads right after the merge), h38 (hook 3 forced to 8 waves/SIMD),
# head (the last commit); one CPU-hour segment in the background.   usage: ab4.sh <tag> <cpu start>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05l}
mkdir -p $O
CPU_PID=
if [ -n "$2" ]; then
  timeout -k 10 1000 python3 -u scripts/cpu_hour.py --cluster 13722 --start $2 --ticks 25 \
    --out $O/cpu_hour_seg$2.jsonl > $O/cpu_hour_seg$2.log 2>&1 &
  CPU_PID=$!
fi
fail() { echo "$1"; [ -n "$CPU_PID" ] && kill $CPU_PID; exit 1; }
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PT tests/test_gpu_band_fast.py tests/test_gpu_scaled.py tests/test_gpu_sharded.py -m gpu > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; fail "tests failed"; }
tail -2 $O/gpu_tests.txt
for k in 1 2; do
  timeout -k 10 300 python3 bench.py --no-cpu --no-pmc --no-companion > $O/sa_h3_$k.json 2> $O/sa_h3_$k.err || fail "bench tree"
  for v in b1 b1kp0 b2h0 h1 h38 head; do
    GM_AB_BUILD=1 GM_LIBRARY=var_fast/libgm_$v.so timeout -k 10 300 python3 bench.py --no-cpu --no-pmc --no-companion > $O/sa_${v}_$k.json 2> $O/sa_${v}_$k.err || fail "bench $v"
  done
done
for f in $O/sa_*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f', round(d['roofline']['kernel_ms'],3), round(d['ms_per_step'],3), round(d['value']/1e6,2))"; done
timeout -k 10 300 python -u scripts/tick_times.py 65536 > $O/tick_times_h3.txt 2>&1 || fail "ticks"
GM_AB_BUILD=1 GM_LIBRARY=var_fast/libgm_head.so timeout -k 10 300 python -u scripts/tick_times.py 65536 > $O/tick_times_head.txt 2>&1 || fail "ticks head"
timeout -k 10 300 python3 scripts/shard_profile.py --sb > $O/sb_stub.json 2> $O/sb_stub.err || fail "sb stub"
timeout -k 10 300 python3 scripts/shard_profile.py --sb --cluster 65536 > $O/sa_stub.json 2> $O/sa_stub.err || fail "sa stub"
GM_SCHUNKS=2 timeout -k 10 300 python3 scripts/shard_profile.py --sb > $O/sb_stub_k2.json 2> $O/sb_stub_k2.err || fail "sb stub k2"
GM_SCHUNKS=8 timeout -k 10 300 python3 scripts/shard_profile.py --sb > $O/sb_stub_k8.json 2> $O/sb_stub_k8.err || fail "sb stub k8"
for f in $O/s?_stub*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f', round(d['ms_per_tick'],3), round(d['band_kernel_ms'],3))"; done
paste $O/tick_times_h3.txt $O/tick_times_head.txt | cut -c1-90 | head -45
if [ -n "$CPU_PID" ]; then wait $CPU_PID; echo "cpu segment rc=$?"; tail -2 $O/cpu_hour_seg$2.jsonl; fi
