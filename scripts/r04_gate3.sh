#!/bin/bash
# round-4 gate after the band fast path: full GPU suite, smoke, the default bench (live PMC traffic,
# S-B companion, CPU baseline), S-C, S-B alone, and the rocprof kernel statistics of S-A
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
bash scripts/gpu.sh r04zp tests smoke sa sc sb prof_sa ticks || exit 1
