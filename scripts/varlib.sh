#!/bin/bash
# measurement-only library variants: varlib/NAME/libgm.so = gm_scaled.hip built with the given -D
# flags, linked with the in-tree build's other objects (run `make` first). usage: varlib.sh NAME -DFLAG...
set -e
cd "$(dirname "$0")/.."
V=$1; shift
mkdir -p build_var/$V varlib/$V
B=distributed-membership_amd/build
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude -Idistributed-membership_amd/csrc "$@" \
  -c -o build_var/$V/gm_scaled.o distributed-membership_amd/csrc/gm_scaled.hip
/opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared -o varlib/$V/libgm.so $B/gm_faithful.o build_var/$V/gm_scaled.o \
  $B/gm_partial.o $B/gm_host.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
