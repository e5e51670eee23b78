#!/bin/bash
# round-4 gate, call 1: the full GPU test suite, smoke, the three bench lines (S-A default with
# live PMC traffic, the S-B companion and the CPU baseline; S-C; S-B on one GPU), the G = 8
# loopback profiles (S-C row shards on one stream, S-B and S-A column shards), and beside them on
# one host core the SCALED restatement for 100 ticks at N = 6,144 (north_star's CPU baseline,
# measured rather than extrapolated; CPU only, joined at the end)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04g
mkdir -p $O
timeout -k 10 1100 python -u scripts/cpu_hour.py --cluster 6144 --ticks 100 --out $O/cpu100_n6144.jsonl \
  > $O/cpu100.log 2>&1 &
CPID=$!
fail() { kill $CPID 2>/dev/null; exit 1; }
bash scripts/gpu.sh r04g tests smoke sa sc sb || fail
timeout -k 10 300 python -u scripts/partial_shard_profile.py > $O/pshard_g8.json 2> $O/pshard_g8.err || fail
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_pshard -o ps -- \
  python3 scripts/partial_shard_profile.py --ticks 4 > $O/prof_pshard.log 2>&1 || fail
timeout -k 10 300 python -u scripts/sb_loopback_profile.py > $O/sb_loopback_g8.json 2> $O/sb_loopback_g8.err || fail
timeout -k 10 200 python -u scripts/sb_loopback_profile.py --cluster 65536 > $O/sa_loopback_g8.json \
  2> $O/sa_loopback_g8.err || fail
wait $CPID
