#!/bin/bash
# Column-shard changes: the shard / limits / band-fast / full-size GPU tests, then the S-A and S-B stub
# shards (gm_shard_stub) under rocprofv3 --kernel-trace --stats.
# usage: scripts/r06/shard_gate.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_sharded.py tests/test_gpu_limits.py tests/test_gpu_band_fast.py tests/test_gpu_gloo_shards.py \
  tests/test_gpu_fullsize_shards.py > $O/gpu_tests.txt 2>&1 || { tail -5 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sashard -o s -- \
  python3 scripts/shard_profile.py --sb --cluster 65536 > $O/sa_stub.json 2> $O/sa_stub.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sbshard -o s -- \
  python3 scripts/shard_profile.py --sb > $O/sb_stub.json 2> $O/sb_stub.err
rc=$?
cut -c1-400 $O/sa_stub.json $O/sb_stub.json
exit $rc
