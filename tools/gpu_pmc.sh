#!/bin/bash
# PMC passes (one counter group per rocprofv3 run; kernel-trace only, no sys-trace).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
B=${1:-4096}
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES" \
           "SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_SALU" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE GRBM_COUNT" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  echo "=== pass $i: $grp"
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc/p$i -o run -- python3 tools/prof_fused.py $B 50 > gpurun_out/pmc/p$i.log 2>&1
  rc=$?
  echo "rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/pmc/p$i.log; exit $rc; fi
done
echo done
