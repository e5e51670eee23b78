#!/bin/bash
# the mt19937 init step's 32-bit multiply: v_mul_lo_u32 against a 24-bit-multiply decomposition
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${1:-r05z}
mkdir -p $O
timeout -k 10 120 ./scripts/ubench/mul32 > $O/mul32.txt 2>&1; rc=$?
cat $O/mul32.txt
exit $rc
