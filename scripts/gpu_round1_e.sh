#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1 &&
timeout -k 10 300 rocprofv3 --selected-regions --kernel-trace --stats -d gpurun_out/prof_sel -o r01 --output-format csv -- python3 bench.py > gpurun_out/prof_sel.log 2>&1 &&
GM_DEVICE_OVERRIDE=0 timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --cluster 4096 --steps 5 --warmup 1 --prologue 12 --crash-tick 5 --no-cpu > gpurun_out/two_rank.log 2>&1
rc=$?
echo "rc=$rc"; tail -n 3 gpurun_out/t_all.log; grep metric gpurun_out/prof_sel.log; tail -n 20 gpurun_out/two_rank.log
exit $rc
