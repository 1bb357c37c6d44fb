set -u
mkdir -p gpurun_out
# degree sets of the config-2 forward (LV_TILE_MASKS, one hex mask per wave): the planner's
# cost-balanced sets, degree 0 moved off the 3-degree wave, LPT over the timeline's per-degree
# times, pairs summing to 10
timeout -k 10 600 bash tools/gpu_variants.sh "--batch 4096 --lmax 10 --dtype f32 --sweep=65536" plan= mv0=LV_TILE_MASKS=400:201:102:84:48:30 lpt=LV_TILE_MASKS=400:201:104:12:88:60 pairs=LV_TILE_MASKS=400:202:104:88:50:21 plan2= mv0b=LV_TILE_MASKS=400:201:102:84:48:30 > gpurun_out/ab_masks_c2.log 2>&1; echo masks rc=$?; cat gpurun_out/ab_masks_c2.log
