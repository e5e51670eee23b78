#!/bin/bash
# Measurement builds of libgm with parts of the PARTIAL tick switched off (GM_P_ABL bits,
# see gm_partial.hip) or the per-section clock build (GM_P_PROFILE), into
# build_var/<name>/libgm.so; run with GM_LIBRARY=build_var/<name>/libgm.so python bench.py ...
# Usage: scripts/sc_variants.sh name:FLAGS ...   e.g. noevict:-DGM_P_ABL=1
set -e
cd "$(dirname "$0")/.."
HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude -Idistributed-membership_amd/csrc -Wno-unused-result"
C=distributed-membership_amd/csrc
B=distributed-membership_amd/build
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  mkdir -p build_var/$name
  /opt/rocm/bin/hipcc $HIPFLAGS $flags -c -o build_var/$name/gm_partial.o $C/gm_partial.hip
  /opt/rocm/bin/hipcc $HIPFLAGS -shared -o build_var/$name/libgm.so $B/gm_faithful.o $B/gm_scaled.o \
    build_var/$name/gm_partial.o $B/gm_host.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
  echo "built build_var/$name/libgm.so ($flags)"
done
