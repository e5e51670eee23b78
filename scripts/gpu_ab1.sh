#!/bin/bash
# A/B: payload plane layout (separate vs row-interleaved) x non-temporal table streams
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_scaled.py tests/test_gpu_sharded.py -x -q --timeout 120 --timeout-method thread -k "64 or 256" > gpurun_out/t_ab.log 2>&1 &&
for cfg in "GM_MSG_SEPARATE=1 GM_NT=0" "GM_MSG_SEPARATE=0 GM_NT=0" "GM_MSG_SEPARATE=0 GM_NT=1" "GM_MSG_SEPARATE=1 GM_NT=1" "GM_MSG_SEPARATE=0 GM_NT=0"; do
  env $cfg timeout -k 10 200 python -u bench.py --no-cpu --steps 30 > gpurun_out/ab.json 2>&1 || exit 1
  echo "$cfg $(python3 -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['achieved'])")"
done
