#!/bin/bash
# round 5 closing gate, part B: the profiles of the final tree -- S-C bench, the S-B / S-A stub shards,
# the G = 8 pipelined S-B loopback, the S-C row-shard loopback (+ its rocprof stats), rocprof stats of
# S-A and S-C, per-tick S-A times, and the SQ instruction mixes of S-A and S-C.
#   usage: scripts/r05/gate_final_b.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-r05q}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_band_fast.py -m gpu > $O/band_fast_tests.txt 2>&1 || { tail -30 $O/band_fast_tests.txt; exit 1; }
tail -2 $O/band_fast_tests.txt
bash scripts/gpu.sh $TAG sc || exit 1
timeout -k 10 300 python3 scripts/shard_profile.py --sb > $O/sb_stub.json 2> $O/sb_stub.err || exit 1
timeout -k 10 300 python3 scripts/shard_profile.py --sb --cluster 65536 > $O/sa_stub.json 2> $O/sa_stub.err || exit 1
timeout -k 10 600 python3 scripts/sb_loopback_profile.py --pipelined > $O/sb_loopback_pipe.json 2> $O/sb_loopback_pipe.err || exit 1
timeout -k 10 300 python3 scripts/partial_shard_profile.py > $O/pshard.json 2> $O/pshard.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_pshard -o ps -- python3 scripts/partial_shard_profile.py --ticks 6 > $O/prof_pshard.log 2>&1 || exit 1
bash scripts/gpu.sh $TAG prof_sa ticks prof_sc mix_sa mix_sc || exit 1
for f in $O/sb_stub.json $O/sa_stub.json $O/sb_loopback_pipe.json $O/pshard.json; do cut -c1-300 $f; done
python3 -c "import json;d=json.load(open('$O/bench_sc.json'));print('S-C', round(d['value']/1e6,1), d['roofline']['kernel_ms'])"
