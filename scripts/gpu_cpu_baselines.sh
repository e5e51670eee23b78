#!/bin/bash
# CPU baselines on the GPU box's host (BASELINE.md "CPU-baseline plan"), plus this
# build's ./Application on the three testcases for comparison.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/cpub
timeout -k 10 900 python3 -u scripts/cpu_baselines.py --gpu --sizes 4096,8192,16384 --seconds 8 --out gpurun_out/cpub/cpu_baselines.json > gpurun_out/cpub/log.txt 2>&1
rc=$?
tail -n 30 gpurun_out/cpub/log.txt
exit $rc
