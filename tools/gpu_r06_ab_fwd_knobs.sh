# Config-2 forward (l = 10, 7 waves per block at 4,096 since the round-6 planner) against the
# tile kernel's other A/B knobs: store policy (LV_TILE_WT 0 = nt, 1 = write-through), wave
# priority phases (LV_TILE_PRIO), prologue tasks over all waves (LV_TILE_SPREAD=1).
set -u
mkdir -p gpurun_out
timeout -k 10 800 bash tools/gpu_variants.sh "--batch 4096 --lmax 10 --dtype f32 --sweep=8192,16384" plan= wt0=LV_TILE_WT=0 prio0=LV_TILE_PRIO=0 prio1=LV_TILE_PRIO=1 prio3=LV_TILE_PRIO=3 spread=LV_TILE_SPREAD=1 plan2= > gpurun_out/ab_fwd_knobs.log 2>&1; echo rc=$?; cat gpurun_out/ab_fwd_knobs.log
