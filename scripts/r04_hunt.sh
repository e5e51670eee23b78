#!/bin/bash
# round-4 diagnostics: the full-size S-C single context, views checked for self after every tick
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04y
mkdir -p $O
PYTHONPATH=distributed-membership_amd timeout -k 10 500 python -u scripts/debug/sc_self_hunt.py 2 1 > $O/hunt.txt 2>&1
