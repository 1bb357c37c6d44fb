#!/bin/bash
# Paired-column tile kernel: parity tests, then A/B against the scalar tile kernel and a
# segment-count sweep at the metric size and at large batch (env knobs read by the library).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  grep -E "passed|failed|^\{" "gpurun_out/$name.log" | cut -c1-420
  if [ $rc -ne 0 ]; then tail -n 30 "gpurun_out/$name.log"; exit $rc; fi
}
run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread
for cfg in "LV_TILE_PAIR=0" "LV_TILE_PAIR=1 LV_PAIR_NSEG=4" "LV_TILE_PAIR=1 LV_PAIR_NSEG=5" "LV_TILE_PAIR=1 LV_PAIR_NSEG=6" "LV_TILE_PAIR=1 LV_PAIR_NSEG=7" "LV_TILE_PAIR=1 LV_PAIR_NSEG=8"; do
  for B in 4096 65536; do
    run "ab_${cfg// /_}_B$B" 120 env $cfg python bench.py --batch $B --steps 1000 --warmup 100 --no-cpu-baseline --multistream 1
  done
done
echo "=== done"
