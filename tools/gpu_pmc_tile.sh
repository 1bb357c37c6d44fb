#!/bin/bash
# PMC passes over the tile harness (tools/kbench_tile <n> <reps> 1): one counter group
# per rocprofv3 run, each under its own time limit.
set -u
cd "$(dirname "$0")/.."
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
N=${1:-4096}; TAG=${2:-tile}; KNAME=${3:-action_fwd_tile}
mkdir -p gpurun_out/pmc_$TAG
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_INSTS_BRANCH" \
           "SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_IFETCH SQ_WAIT_INST_LDS" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ SQC_TC_INST_REQ SQC_TC_STALL" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT" \
           "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc_$TAG/p$i -o run -- ./tools/kbench_tile $N 50 1 > gpurun_out/pmc_$TAG/p$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pass $i rc=$rc"; tail -5 gpurun_out/pmc_$TAG/p$i.log; exit $rc; fi
done
python3 tools/pmc_summary.py gpurun_out/pmc_$TAG $KNAME
