#!/bin/bash
# The one GPU-box runner: every committed profile under profiles/rNN/ names the
# tag and step list it came from (`scripts/gpu.sh <tag> <step>...`).
#
#   tests      python -m pytest tests -m gpu            -> $O/gpu_tests.txt
#   smoke      __graft_entry__.smoke()                  -> $O/smoke.txt
#   sa         bench.py (S-A, with cpu_baseline, live PMC traffic and the S-B companion run) -> $O/bench_sa.json
#   sc         bench.py --scenario S-C                  -> $O/bench_sc.json
#   ticks      scripts/tick_times.py: per-tick gm_s_band time of the S-A schedule -> $O/tick_times.txt
#   sb         bench.py --cluster 262144 (S-B on one GPU) -> $O/bench_sb.json
#   sa_pmc     bench.py --pmc (S-A, traffic measured live by two child PMC passes) -> $O/bench_sa_pmc.json
#   shard      bench.py --force-shard (RCCL, 1 rank)    -> $O/bench_force_shard.json
#   sbshard    scripts/shard_profile.py --sb            -> $O/sb_shard.json
#   prof_sa    rocprofv3 --kernel-trace --stats of S-A  -> $O/prof_sa/
#   prof_sc    rocprofv3 --kernel-trace --stats of S-C  -> $O/prof_sc/
#   prof_sb    rocprofv3 --kernel-trace --stats of S-B (N = 262,144, one GPU) -> $O/prof_sb/
#   pmc_sa     FETCH_SIZE / WRITE_SIZE passes of S-A    -> $O/pmc_sa_{fetch,write}/ + traffic json
#   mix_sa     SQ instruction mix of S-A (one --pmc pass)  -> $O/mix_sa/
#   pmc_sc     FETCH_SIZE / WRITE_SIZE passes of S-C    -> $O/pmc_sc_{fetch,write}/ + traffic json
#   mix_sc     SQ instruction mix / wave-cycle split of S-C (one --pmc pass) -> $O/mix_sc/
#   faithful   ./Application on the three testcases + N = 70, timed -> $O/faithful_wall.txt
#   prof_faithful rocprofv3 --kernel-trace --stats of ./Application at N = 70 -> $O/prof_n70/
#
# Every GPU step runs under its own timeout; steps are chained so the first
# failure ends the call (no retries). Extra bench flags: BENCH_ARGS env.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:?usage: scripts/gpu.sh <tag> <step>...}
shift
O=gpurun_out/$TAG
mkdir -p "$O"
PT="python -u -m pytest -x -v --timeout 150 --timeout-method thread"

run_step() {
  case "$1" in
    tests) timeout -k 10 1400 $PT ${TESTS:-tests} -m gpu --durations 15 > $O/gpu_tests.txt 2>&1 ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 ;;
    sa) timeout -k 10 300 python -u bench.py ${BENCH_ARGS:-} > $O/bench_sa.json 2> $O/bench_sa.err ;;
    sc) timeout -k 10 400 python -u bench.py --scenario S-C ${BENCH_ARGS:-} > $O/bench_sc.json 2> $O/bench_sc.err ;;
    ticks) timeout -k 10 300 python -u scripts/tick_times.py ${TICKS_N:-65536} > $O/tick_times.txt 2>&1 ;;
    sb) timeout -k 10 400 python -u bench.py --cluster 262144 ${BENCH_ARGS:-} > $O/bench_sb.json 2> $O/bench_sb.err ;;
    sa_pmc) timeout -k 10 700 python -u bench.py --pmc --no-cpu ${BENCH_ARGS:-} > $O/bench_sa_pmc.json 2> $O/bench_sa_pmc.err ;;
    shard) timeout -k 10 300 python -u bench.py --force-shard --no-cpu --no-pmc --no-companion ${BENCH_ARGS:-} > $O/bench_force_shard.json 2> $O/bench_force_shard.err ;;
    sbshard) timeout -k 10 400 python -u scripts/shard_profile.py --sb > $O/sb_shard.json 2> $O/sb_shard.err ;;
    prof_sa) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sa -o sa -- \
               python3 bench.py --no-cpu --no-pmc --no-companion ${BENCH_ARGS:-} > $O/prof_sa.log 2>&1 ;;
    prof_sc) timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sc -o sc -- \
               python3 bench.py --scenario S-C --no-cpu --no-pmc ${BENCH_ARGS:-} > $O/prof_sc.log 2>&1 ;;
    prof_sb) timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sb -o sb -- \
               python3 bench.py --cluster 262144 --no-cpu --no-pmc ${BENCH_ARGS:-} > $O/prof_sb.log 2>&1 ;;
    pmc_sa) timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_sa_fetch -o p -- \
              python3 bench.py --no-cpu --no-pmc --no-companion --steps 5 --warmup 1 > $O/pmc_sa_fetch.log 2>&1 &&
            timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_sa_write -o p -- \
              python3 bench.py --no-cpu --no-pmc --no-companion --steps 5 --warmup 1 > $O/pmc_sa_write.log 2>&1 &&
            python3 scripts/pmc_traffic.py --kernel gm_s_band --fetch $O/pmc_sa_fetch --write $O/pmc_sa_write \
              --layout byte-band --out $O/traffic_n65536.json > $O/pmc_sa.txt 2>&1 ;;
    mix_sa) timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY \
              --kernel-trace --output-format csv -d $O/mix_sa -o p -- python3 bench.py --no-cpu --no-pmc --no-companion --steps 5 --warmup 1 > $O/mix_sa.log 2>&1 ;;
    mix_sc) timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
              --kernel-trace --output-format csv -d $O/mix_sc -o p -- python3 bench.py --scenario S-C --no-cpu --no-pmc --steps 3 --warmup 1 > $O/mix_sc.log 2>&1 ;;
    pmc_sc) timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_sc_fetch -o p -- \
              python3 bench.py --scenario S-C --no-cpu --no-pmc --steps 3 --warmup 1 > $O/pmc_sc_fetch.log 2>&1 &&
            timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_sc_write -o p -- \
              python3 bench.py --scenario S-C --no-cpu --no-pmc --steps 3 --warmup 1 > $O/pmc_sc_write.log 2>&1 &&
            python3 scripts/pmc_traffic.py --kernel gm_p_tick --fetch $O/pmc_sc_fetch --write $O/pmc_sc_write \
              --layout partial-v32 --n 16777216 --out $O/traffic_sc_n16777216.json > $O/pmc_sc.txt 2>&1 ;;
    faithful) ( TIMEFORMAT="%R s"; for c in singlefailure multifailure msgdropsinglefailure n70; do
                  echo -n "$c "; { time timeout -k 10 60 ./Application testcases/$c.conf > /dev/null; } 2>&1 || exit 1
                done ) > $O/faithful_wall.txt 2>&1 ;;
    prof_faithful) timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_n70 -o n70 -- \
               ./Application testcases/n70.conf > $O/prof_n70.log 2>&1 ;;
    *) echo "unknown step $1"; return 2 ;;
  esac
}

rc=0
for s in "$@"; do
  echo "[$(date +%T)] step $s" | tee -a $O/steps.txt
  run_step "$s" || { rc=$?; echo "step $s failed rc=$rc" | tee -a $O/steps.txt; break; }
done
echo "rc=$rc"
for f in $O/gpu_tests.txt $O/smoke.txt; do [ -f $f ] && tail -n 3 $f; done
for f in $O/*.json; do [ -f $f ] && cut -c1-400 $f; done
exit $rc
