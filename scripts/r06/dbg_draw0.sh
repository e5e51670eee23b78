#!/bin/bash
# Diagnostics: the column-shard band-fast test with a libgm that prints every gm_s_draw0 draw no lane
# holds (build_dbg/libgm.so: this tree's gm_scaled.hip plus one printf), then gate A.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r06b
GM_AB_BUILD=1 GM_LIBRARY=build_dbg/libgm.so timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread \
  tests/test_gpu_band_fast.py -m gpu -k column_shards > gpurun_out/r06b/dbg.txt 2>&1
echo "dbg rc=$?"
grep -c NOHOLDER gpurun_out/r06b/dbg.txt
grep NOHOLDER gpurun_out/r06b/dbg.txt | head -20
bash scripts/r06/gate_a.sh r06b
