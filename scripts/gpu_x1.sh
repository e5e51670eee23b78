#!/bin/bash
# EXPERIMENT: payload-read locality (sender id masked) vs band kernel time.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in 0 63 4095 16383; do
 for b in 128 512; do
  GM_XMASK=$m GM_BAND=$b timeout -k 10 200 python -u bench.py --no-cpu --steps 8 --warmup 1 --prologue 9 > gpurun_out/x_${m}_${b}.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/x_${m}_${b}.log').read().strip().splitlines()[-1]); print('mask $m band $b', round(d['roofline']['kernel_ms'],2))"
 done
done
