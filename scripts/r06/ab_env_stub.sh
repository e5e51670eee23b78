#!/bin/bash
# Interleaved stub-shard runs (S-A: N = 65,536, rank 3 of 8) under environment variants.
# usage: scripts/r06/ab_env_stub.sh <tag> "<ENV=..>" "<ENV=..>" ...   ("-" = no extra env)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${1:?tag}; shift; mkdir -p $O
for i in 1 2 3; do
  k=0
  for e in "$@"; do
    k=$((k + 1))
    [ "$e" = - ] && e=""
    env $e timeout -k 10 200 python3 scripts/shard_profile.py --sb --cluster ${STUB_N:-65536} > $O/v${k}_$i.json 2>/dev/null || exit 1
  done
done
k=0
for e in "$@"; do k=$((k + 1)); for f in $O/v${k}_*.json; do python3 -c "
import json; d=json.load(open('$f')); print('$e', '$f', round(d['ms_per_tick'],4), round(d['band_kernel_ms'],4), d['err'])"; done; done
