#!/bin/bash
# Diagnostics (run at round 6 with profiles/r06/stub_tail/diag_nowait.patch applied; the toggle is not in
# the product): the S-A stub shard tick with and without the host's settle wait (GM_DIAG_NOWAIT=1:
# timing only), plus a kernel trace of the no-wait run. usage: scripts/r06/stub_nowait.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:?tag}; mkdir -p $O
for i in 1 2; do
  timeout -k 10 200 python3 scripts/shard_profile.py --sb --cluster 65536 > $O/wait_$i.json 2>/dev/null || exit 1
  GM_DIAG_NOWAIT=1 timeout -k 10 200 python3 scripts/shard_profile.py --sb --cluster 65536 > $O/nowait_$i.json 2>/dev/null || exit 1
done
GM_DIAG_NOWAIT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_nowait -o s -- \
  python3 scripts/shard_profile.py --sb --cluster 65536 > $O/nowait_prof.json 2>/dev/null || exit 1
for f in $O/*.json; do python3 -c "
import json; d=json.load(open('$f')); print('$f', round(d['ms_per_tick'],4), round(d['band_kernel_ms'],4), d['err'])"; done
