#!/bin/bash
# S-C at G = 8 row shards on one device (loopback): per-shard kernel times + exchange volume.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/y
timeout -k 10 400 python3 -u scripts/partial_shard_profile.py > gpurun_out/y/profile.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/y/trace -o sc8 --output-format csv -- python3 scripts/partial_shard_profile.py --ticks 4 > gpurun_out/y/trace.log 2>&1
rc=$?
echo "rc=$rc"; tail -n 2 gpurun_out/y/profile.log; find gpurun_out/y/trace -name '*kernel_stats.csv' -exec cat {} \;
exit $rc
