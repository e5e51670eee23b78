#!/bin/bash
# Build libgm.so from the current csrc with patches applied into build_dbg/<name>/ (A/B scratch;
# the product library is untouched). usage: scripts/r06/build_variant.sh <name> [patch ...]
# EXTRA_FLAGS: more hipcc flags (e.g. -DGM_FAST_WG=1). A patch named "w7" sets the S-C node kernel to amdgpu_waves_per_eu(7, 8).
set -e
N=${1:?name}; shift
cd "$(dirname "$0")/../.."
W=/tmp/var_$N
rm -rf $W && mkdir -p $W/csrc $W/obj && cp distributed-membership_amd/csrc/* $W/csrc/
for p in "$@"; do
  if [ "$p" = w7 ]; then
    sed -i 's/amdgpu_waves_per_eu(8, 8))) void gm_p_tick_small_pf/amdgpu_waves_per_eu(7, 8))) void gm_p_tick_small_pf/' $W/csrc/gm_partial.hip
    grep -q "amdgpu_waves_per_eu(7, 8))) void gm_p_tick_small_pf" $W/csrc/gm_partial.hip
  else
    patch -s -d $W/csrc -p3 < "$p"
  fi
done
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude -I$W/csrc -Wall -Wno-unused-result -Wno-pass-failed ${EXTRA_FLAGS:-}"
for k in gm_faithful gm_scaled gm_partial gm_host; do /opt/rocm/bin/hipcc $F -c -o $W/obj/$k.o $W/csrc/$k.hip & done
wait
mkdir -p build_dbg/$N
/opt/rocm/bin/hipcc $F -shared -o build_dbg/$N/libgm.so $W/obj/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built build_dbg/$N/libgm.so
