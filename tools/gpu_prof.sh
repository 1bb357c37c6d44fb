#!/bin/bash
# rocprofv3 evidence for one bench configuration: kernel-trace stats, then separate PMC
# passes (FETCH_SIZE, WRITE_SIZE, two SQ groups), then the HBM-traffic JSON the bench
# line reads (profiles/traffic_B<B>_L<L>_C<C>_<dtype>.json is copied by hand).
#   bash tools/gpu_prof.sh <tag> <bench args...>
# e.g. bash tools/gpu_prof.sh c2 --batch 4096 --lmax 10 --dtype f32
set -u
cd "$(dirname "$0")/.."
TAG=$1; shift
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
BENCH="bench.py --no-cpu-baseline --cold-launches 0 --multistream 1 --no-fwd-bwd --config5-launches 0 --train-steps 0 --sweep= $*"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -s KILL "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 5 "$OUT/$name.log"; echo "stopping"; exit $rc; fi
}
run stats 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- python3 $BENCH --steps 300 --warmup 50
rm -f "$OUT"/stats/*kernel_trace.csv
run fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_tr/fetch" -o run -- python3 $BENCH --steps 100 --warmup 20 --launch eager
run write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_tr/write" -o run -- python3 $BENCH --steps 100 --warmup 20 --launch eager
run sq1 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d "$OUT/pmc/sq1" -o run -- python3 $BENCH --steps 100 --warmup 20 --launch eager
run sq2 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$OUT/pmc/sq2" -o run -- python3 $BENCH --steps 100 --warmup 20 --launch eager
python3 tools/pmc_traffic.py "$OUT/pmc_tr" "$OUT/traffic.json"
python3 tools/pmc_summary.py "$OUT/pmc" action_fwd > "$OUT/pmc_summary.txt"
find "$OUT" -name "*counter_collection.csv" -size +2M -delete
cat "$OUT/pmc_summary.txt"
echo "=== done"
