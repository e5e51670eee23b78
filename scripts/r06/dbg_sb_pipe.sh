#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r06c
GM_AB_BUILD=1 GM_LIBRARY=build_dbg/libgm.so timeout -k 10 400 python3 -u scripts/r06/dbg_sb_pipe.py > gpurun_out/r06c/sb_pipe.txt 2>&1
echo "rc=$?"
tail -5 gpurun_out/r06c/sb_pipe.txt
