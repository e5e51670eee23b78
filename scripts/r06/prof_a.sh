#!/bin/bash
# Round 6 profiles: (1) one S-A column shard alone (gm_shard_stub, rank 3 of 8: 8,192 columns) and one
# S-B shard under rocprofv3 --kernel-trace --stats, to split the per-tick non-band work by kernel;
# (2) the S-A SQ mix per dispatch over the whole bench window (ticks 9..48, incl. the TREMOVE peak);
# (3) S-A per-tick band-kernel times.
# usage: scripts/r06/prof_a.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sashard -o s -- \
  python3 scripts/shard_profile.py --sb --cluster 65536 > $O/sa_stub.json 2> $O/sa_stub.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sbshard -o s -- \
  python3 scripts/shard_profile.py --sb > $O/sb_stub.json 2> $O/sb_stub.err &&
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY \
  --kernel-trace --output-format csv -d $O/mix_sa -o p -- python3 bench.py --no-cpu --no-pmc --no-companion > $O/mix_sa.log 2>&1 &&
timeout -k 10 300 python3 -u scripts/tick_times.py 65536 > $O/tick_times.txt 2>&1
rc=$?
echo "rc=$rc"
cat $O/sa_stub.json $O/sb_stub.json
exit $rc
