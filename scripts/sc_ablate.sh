#!/bin/bash
# GPU-box step: S-C bench per measurement build of scripts/sc_variants.sh (build_var/<name>/libgm.so)
# VARIANTS="name ..." (default: the in-tree library only, as "main"); results in gpurun_out/abl/
set -o pipefail
mkdir -p gpurun_out/abl
for v in ${VARIANTS:-main}; do
  echo "[$(date +%T)] $v" >> gpurun_out/abl/steps.txt
  lib=build_var/$v/libgm.so; [ "$v" = main ] && lib=distributed-membership_amd/lib/libgm.so
  GM_AB_BUILD=1 GM_LIBRARY=$lib timeout -k 10 150 python -u bench.py --scenario S-C --no-cpu --no-pmc --steps 10 --warmup 2 \
    > gpurun_out/abl/$v.json 2> gpurun_out/abl/$v.err; rc=$?; echo "$v rc=$rc" >> gpurun_out/abl/steps.txt; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && exit 1
done
exit 0
