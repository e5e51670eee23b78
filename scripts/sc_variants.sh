#!/bin/bash
# Measurement builds of libgm (e.g. the per-section clock build: apply
# profiles/r06/profile_patches/gm_p_profile.patch, then -DGM_P_PROFILE; or a candidate
# kernel change kept beside the in-tree library for an A/B timing) into
# build_var/<name>/libgm.so; run with GM_AB_BUILD=1 GM_LIBRARY=build_var/<name>/libgm.so python bench.py ...
# Usage: scripts/sc_variants.sh name:FLAGS ...   e.g. prof:-DGM_P_PROFILE
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
