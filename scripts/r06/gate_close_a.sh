#!/bin/bash
# Round 6 closing gate, part A: the whole GPU suite, smoke, the S-A headline (live PMC traffic,
# cpu_baseline, S-B companion), S-C, S-B alone on one GPU, live S-C PMC traffic.
# usage: scripts/r06/gate_close_a.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
bash scripts/gpu.sh ${1:?tag} tests smoke sa sc sb pmc_sc
