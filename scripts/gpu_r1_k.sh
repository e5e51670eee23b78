#!/bin/bash
# packed narrow-cell band kernel: SCALED + sharded parity, bench A/B, SQ counters at B=512.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_scaled.py tests/test_gpu_sharded.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_scaled.log 2>&1 &&
for b in 128 256 512; do GM_BAND=$b timeout -k 10 200 python -u bench.py --no-cpu > gpurun_out/bench_b$b.log 2>&1 || exit 1; done &&
GM_BAND=512 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pks -o r --output-format csv -- python3 bench.py --no-cpu > gpurun_out/pks.log 2>&1 &&
GM_BAND=512 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY --kernel-trace --output-format csv -d gpurun_out/pkc -o r -- python3 bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/pkc.log 2>&1
rc=$?
echo "rc=$rc"; tail -n 2 gpurun_out/t_scaled.log
for b in 128 256 512; do python3 -c "import json; d=json.loads(open('gpurun_out/bench_b$b.log').read().strip().splitlines()[-1]); print('b$b', round(d['value']), round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3))" 2>/dev/null || tail -3 gpurun_out/bench_b$b.log; done
python3 - <<'PY'
import csv,collections
d=collections.defaultdict(list)
try:
    for r in csv.DictReader(open('gpurun_out/pkc/r_counter_collection.csv')):
        if 'band' in r['Kernel_Name']: d[r['Counter_Name']].append(float(r['Counter_Value']))
    for k,v in d.items(): print(k, f'{v[-1]:.3g}')
except Exception as e: print(e)
PY
cat gpurun_out/pks/r_kernel_stats.csv
exit $rc
