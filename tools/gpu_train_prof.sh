#!/bin/bash
# Steady-state profile of the config-3 training step (one GPU, B = 512): MIOpen's find
# runs in a separate PRIOR process that fills the user find-db; the timed and profiled
# processes run with --no-find (immediate mode), which takes each convolution's solution
# from that find-db record -- no search, so no naive_conv verification kernels in the
# trace (with find enabled every new process searches again).  Per variant: the timing
# JSON with and without find, a rocprofv3 kernel-trace (--stats) and one PMC pass for
# MFMA utilisation per kernel.
#   bash tools/gpu_train_prof.sh [variant ...]   variants: f32 bf16 f32_nogemm bf16_nogemm bf16_transposed
#   bf16_norelu bf16_miodgrad bf16_foreach
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/train_prof
mkdir -p "$OUT/miopen_db" "$OUT/miopen_cache"
export MIOPEN_USER_DB_PATH="$PWD/$OUT/miopen_db" MIOPEN_CUSTOM_CACHE_DIR="$PWD/$OUT/miopen_cache"
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 2 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
VARIANTS=${*:-f32 bf16}
for v in $VARIANTS; do
  case $v in
    f32) A="" ;;
    bf16) A="--amp bf16 --channels-last" ;;
    f32_nogemm) A="--conv-gemm off" ;;
    bf16_nogemm) A="--amp bf16 --channels-last --conv-gemm off" ;;
    bf16_transposed) A="--amp bf16 --channels-last --deconv transposed" ;;
    bf16_norelu) A="--amp bf16 --channels-last --fused-relu off" ;;
    bf16_miodgrad) A="--amp bf16 --channels-last --conv-dgrad miopen" ;;
    bf16_foreach) A="--amp bf16 --channels-last --adam foreach" ;;
    *) echo "unknown variant $v"; exit 2 ;;
  esac
  step warm_$v 600 python bench_train.py --steps 3 --warmup 2 $A
  step time_$v 300 python bench_train.py --steps 30 --warmup 5 $A
  step timedb_$v 300 python bench_train.py --steps 30 --warmup 5 --no-find $A
  if [ "${TIMEONLY:-0}" = 1 ]; then continue; fi
  ( cd /tmp && export TMPDIR=/tmp )
  export TMPDIR=/tmp
  # 3 warm-up + 1 FLOP-count + 20 timed steps
  step stats_$v 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats_$v" -o run --output-format csv -- python3 bench_train.py --steps 20 --warmup 3 --no-find $A
  rm -f "$OUT"/stats_$v/*kernel_trace.csv
  step pmc_$v 300 timeout -s KILL 280 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_$v" -o run -- python3 bench_train.py --steps 3 --warmup 1 --no-find $A
  python3 tools/train_kernel_table.py "$OUT/stats_$v/run_kernel_stats.csv" 24 "$OUT/pmc_$v" > "$OUT/table_$v.txt"
  find "$OUT/pmc_$v" -name "*counter_collection.csv" -size +4M -delete
  head -25 "$OUT/table_$v.txt"
done
echo "=== done"
