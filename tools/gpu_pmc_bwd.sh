#!/bin/bash
# PMC passes (one counter group per run) on the config-2 training direction: the bench's
# fwd_bwd leg runs the fused forward, the backward tile kernel and the dF reduce.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/pmc_bwd
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
BENCH="bench.py --steps 20 --warmup 5 --no-cpu-baseline --cold-launches 0 --multistream 1 --launch eager"
i=0
for g in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
         "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $g --output-format csv -d "$OUT/p$i" -o run -- python3 $BENCH > "$OUT/p$i.log" 2>&1 || { echo "pass $i rc=$?"; tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 tools/pmc_summary.py "$OUT" action_bwd_tile > "$OUT/summary_bwd_tile.txt"
python3 tools/pmc_summary.py "$OUT" action_bwd_reduce > "$OUT/summary_bwd_reduce.txt"
python3 tools/pmc_summary.py "$OUT" action_fwd_tile > "$OUT/summary_fwd_tile.txt"
find "$OUT" -name "*counter_collection.csv" -size +2M -delete
cat "$OUT/summary_bwd_tile.txt" "$OUT/summary_bwd_reduce.txt" "$OUT/summary_fwd_tile.txt"
echo done
