#!/bin/bash
# round 5: S-C row shards with the records built by gm_p_pack from targets + lists -- PARTIAL tests,
# then the G = 8 loopback of N = 16M (rocprof kernel stats)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05i}
mkdir -p $O
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PT tests/test_gpu_partial.py tests/test_gpu_fullsize_shards.py tests/test_gpu_msgcount.py -m gpu \
  > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -3 $O/gpu_tests.txt
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_pshard -o p -- \
  python3 scripts/partial_shard_profile.py > $O/pshard_g8.json 2> $O/pshard_g8.err
rc=$?
cat $O/pshard_g8.json
python3 - <<'PY' $O/prof_pshard/p_kernel_stats.csv
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"{r['Name'][:60]:60s} calls={r['Calls']:>5} avg_us={float(r['AverageNs'])/1e3:9.2f} tot_ms={float(r['TotalDurationNs'])/1e6:9.2f}")
PY

[ $rc -eq 0 ] || exit $rc
# the S-A headline: this tree's library against round 4's final one (var_ab/libgm_r04.so), interleaved
for k in 1 2; do
  timeout -k 10 300 python3 bench.py --no-cpu --no-pmc --no-companion > $O/sa_cur_$k.json 2> $O/sa_cur_$k.err || exit 1
  GM_AB_BUILD=1 GM_LIBRARY=var_ab/libgm_r04.so timeout -k 10 300 python3 bench.py --no-cpu --no-pmc --no-companion > $O/sa_r04_$k.json 2> $O/sa_r04_$k.err || exit 1
done
for f in $O/sa_*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f', round(d['roofline']['kernel_ms'],3), round(d['ms_per_step'],3), round(d['value']/1e6,2))"; done
