# Backward at 4,096 / 8,192 (persistent kernel + reduce5): grid size (LV_BWD_PERSIST_BPC:
# 1 / 2 blocks per CU -> fewer dF slabs, more groups per block) against the default
# (3 per CU: one group per block at 4,096), backward alone (tools/bwd_reduce_ab.py).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_KNOBS="LV_BWD_PERSIST_BPC=3,LV_BWD_PERSIST_BPC=1,LV_BWD_PERSIST_BPC=2,LV_BWD_PERSIST_BPC=3,LV_BWD_PERSIST_BPC=2" \
  timeout -k 10 600 python -u tools/bwd_reduce_ab.py 4096 8192 > gpurun_out/ab_bwd_small.log 2>&1; echo ab rc=$?; cat gpurun_out/ab_bwd_small.log
