set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/ab_schunks; mkdir -p $O
for i in 1 2; do for k in 2 4 8; do
  GM_SCHUNKS=$k timeout -k 10 200 python3 scripts/shard_profile.py --sb --cluster 65536 > $O/k${k}_$i.json 2>/dev/null || exit 1
  GM_SCHUNKS=$k timeout -k 10 300 python3 scripts/shard_profile.py --sb > $O/sb_k${k}_$i.json 2>/dev/null || exit 1
done; done
for f in $O/*.json; do python3 -c "
import json; d=json.load(open('$f')); print('$f', d['n'], round(d['ms_per_tick'],4), round(d['band_kernel_ms'],4))"; done
