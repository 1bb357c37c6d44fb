#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) on tools/bwd_only.py: the backward alone
# (tile or persistent kernel + dF reduce), graph-replayed, at batch B (default 65536).
#   bash tools/gpu_pmc_bwd_only.sh 65536 action_bwd_persist
set -u
cd "$(dirname "$0")/.."
B=${1:-65536}
K=${2:-action_bwd_persist}
OUT=gpurun_out/pmc_bwd_only_$B
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for g in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
         "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $g --output-format csv -d "$OUT/p$i" -o run -- python3 tools/bwd_only.py $B 2 > "$OUT/p$i.log" 2>&1 || { echo "pass $i rc=$?"; tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 tools/pmc_summary.py "$OUT" $K > "$OUT/summary.txt"
python3 tools/pmc_summary.py "$OUT" action_bwd_reduce > "$OUT/summary_reduce.txt"
find "$OUT" -name "*counter_collection.csv" -size +2M -delete
cat "$OUT/summary.txt" "$OUT/summary_reduce.txt"
echo done
