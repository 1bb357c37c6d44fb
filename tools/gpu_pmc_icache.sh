#!/bin/bash
# Instruction-cache / issue PMC passes over the fused forward at l = 10 and l = 20
# (tools/prof_fused.py).  One counter group per rocprofv3 run, each under its own time
# limit; stops at the first failure.
set -u
cd "$(dirname "$0")/.."
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=gpurun_out/pmc_ic${PMC_TAG:-}
mkdir -p $OUT
run() {  # dir, counters, cmd...
  local d=$1 grp=$2; shift 2
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $d -o run -- "$@" > $d.log 2>&1
  local rc=$?
  echo "$d rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $d.log; exit $rc; fi
}
for L in ${PMC_LS:-10 20}; do
  B=$([ $L = 10 ] && echo 4096 || echo 8192)
  mkdir -p $OUT/L$L
  run $OUT/L$L/a "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" python3 tools/prof_fused.py $B 30 $L 10
  run $OUT/L$L/b "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ SQC_TC_INST_REQ SQC_TC_STALL" python3 tools/prof_fused.py $B 30 $L 10
  run $OUT/L$L/c "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT" python3 tools/prof_fused.py $B 30 $L 10
  python3 tools/pmc_summary.py $OUT/L$L action_fwd > $OUT/summary_L$L.txt 2>&1
done
for f in $OUT/summary_L*.txt; do echo "== $f"; cat $f; done
