#!/bin/bash
# round-4: pack-kernel exchange with single-stream loopback; bench default (live PMC traffic)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04f
mkdir -p $O
TESTS="tests/test_gpu_partial.py tests/test_gpu_fullsize_shards.py" bash scripts/gpu.sh r04f tests || exit 1
timeout -k 10 300 python -u scripts/partial_shard_profile.py > $O/pshard_g8.json 2> $O/pshard_g8.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_pshard -o ps -- \
  python3 scripts/partial_shard_profile.py --ticks 4 > $O/prof_pshard.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $O/bench_sa.json 2> $O/bench_sa.err || exit 1
timeout -k 10 400 python -u scripts/sb_loopback_profile.py > $O/sb_loopback_g8.json 2> $O/sb_loopback_g8.err
