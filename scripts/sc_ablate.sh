set -o pipefail
mkdir -p gpurun_out/abl
for v in base noevict noret norank nodrop all; do
  echo "[$(date +%T)] $v" >> gpurun_out/abl/steps.txt
  GM_LIBRARY=build_var/$v/libgm.so timeout -k 10 150 python -u bench.py --scenario S-C --no-cpu --steps 10 --warmup 2 > gpurun_out/abl/$v.json 2> gpurun_out/abl/$v.err || exit 1
done
