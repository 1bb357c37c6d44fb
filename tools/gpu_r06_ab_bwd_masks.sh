# Degree sets of the persistent backward's 4 waves at l = 10 (LV_BWD_MASKS, A/B library):
# the planner's {10,3} {9,4,0} {8,5,1} {7,6,2} against the best-balanced alternatives
# under other per-degree fixed costs (tools/bwd_reduce_ab.py, backward alone).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_KNOBS="LV_BWD_MASKS=408:211:122:c4,LV_BWD_MASKS=408:211:140:a6,LV_BWD_MASKS=406:211:140:a8,LV_BWD_MASKS=405:240:122:98,LV_BWD_MASKS=410:240:122:8d,LV_BWD_MASKS=408:211:122:c4" \
  timeout -k 10 600 python -u tools/bwd_reduce_ab.py 4096 65536 > gpurun_out/ab_bwd_masks.log 2>&1; echo ab rc=$?; cat gpurun_out/ab_bwd_masks.log
