#!/bin/bash
# round 5: S-C row shards -- parity of the tree's library, then the G = 8 loopback of N = 16M with the
# chunk launches at 4 (tree), 8 and 16 (var_pshard/) nodes per wave
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05k}
mkdir -p $O
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $PT tests/test_gpu_partial.py tests/test_gpu_fullsize_shards.py -m gpu -k "row_shard or packed or half or sc_full" \
  > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -3 $O/gpu_tests.txt
timeout -k 10 300 python3 scripts/partial_shard_profile.py > $O/pshard_npw4.json 2> $O/pshard_npw4.err || exit 1
for v in 8 16; do
  GM_AB_BUILD=1 GM_LIBRARY=var_pshard/libgm_npw$v.so timeout -k 10 300 python3 scripts/partial_shard_profile.py > $O/pshard_npw$v.json 2> $O/pshard_npw$v.err || exit 1
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_pshard -o p -- \
  python3 scripts/partial_shard_profile.py > $O/pshard_prof.json 2> $O/pshard_prof.err
rc=$?
for f in $O/pshard_*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f', round(d['ms_per_tick_all_shards_serialised']/d['shards'],3), d['recv_mb_mean'])"; done
python3 - <<'PY' $O/prof_pshard/p_kernel_stats.csv
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"{r['Name'][:60]:60s} calls={r['Calls']:>5} avg_us={float(r['AverageNs'])/1e3:9.2f} tot_ms={float(r['TotalDurationNs'])/1e6:9.2f}")
PY
exit $rc
