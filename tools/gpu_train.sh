#!/bin/bash
# Config-3 training step on one GPU: default MIOpen solutions, MIOpen find, NHWC + find;
# then MFMA PMC counters over a short run.  Every GPU step has its own time limit and a
# failure ends the script.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/train
mkdir -p $OUT
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 3 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step c3 300 python bench_train.py --steps 20 --no-find
step c3_find 400 python bench_train.py --steps 20
step c3_nhwc_find 400 python bench_train.py --steps 20 --channels-last
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 60 rocprofv3 --list-avail > $OUT/avail.txt 2>&1
grep -o "SQ_[A-Z_]*MFMA[A-Z0-9_]*" $OUT/avail.txt | sort -u > $OUT/mfma_counters.txt
cat $OUT/mfma_counters.txt
CNT=""
for c in SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F32; do
  grep -qx "$c" $OUT/mfma_counters.txt && CNT="$CNT $c"
done
echo "counters:$CNT"
if [ -n "$CNT" ]; then
  step pmc_mfma 300 rocprofv3 --pmc $CNT GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc -o run -- python3 bench_train.py --steps 5 --warmup 2
fi
echo done
