#!/bin/bash
# Round 6 gate A: the whole GPU suite + smoke + the S-A headline (warm start, t0 = 8), then the
# survey's literal S-A start (cold converged start, hb = ts = 0, bench.py --t0 0) beside it.
# usage: scripts/r06/gate_a.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
T=${1:?tag}
bash scripts/gpu.sh $T tests smoke sa &&
BENCH_ARGS="--t0 0 --no-companion" bash scripts/gpu.sh ${T}_cold sa
