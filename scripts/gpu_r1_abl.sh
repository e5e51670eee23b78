#!/bin/bash
# PARTIAL ablations (GM_LIBRARY per variant; each replaces one section by a cheaper,
# statistically equivalent stand-in -- not parity builds): S-C N=16M bench per variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-abl}
mkdir -p $O
rc=0
for v in ${VARIANTS:-d a1 a2 a3}; do
  GM_LIBRARY=distributed-membership_amd/lib/libgm_$v.so timeout -k 10 200 python3 -u bench.py --scenario S-C --no-cpu --steps 10 > $O/bench_$v.json 2> $O/bench_$v.err || { rc=$?; break; }
  python3 -c "import json; d=json.load(open('$O/bench_$v.json')); print('$v', round(d['ms_per_step'],2), round(d['roofline']['kernel_ms'],2))"
done
echo "rc=$rc"
exit $rc
