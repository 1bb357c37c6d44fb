# Degree sets of the config-5 forward (l = 20, 8 waves; LV_TILE_MASKS, A/B library) after
# the forward's fixed per-degree cost moved 40 -> 80: the planner's sets against the
# fixed-cost-40 sets (round-6 start) and the fixed-cost-0 sets; then config 2 at 5 / 7
# waves with the new cost model against the planned 6.
set -u
mkdir -p gpurun_out
timeout -k 10 500 bash tools/gpu_variants.sh "--batch 8192 --lmax 20 --dtype bf16" plan= f40=LV_TILE_MASKS=100008:80040:40080:20101:10202:8404:4810:3020 f0=LV_TILE_MASKS=100002:80040:40080:20101:10204:8408:4810:3020 plan2= f40b=LV_TILE_MASKS=100008:80040:40080:20101:10202:8404:4810:3020 > gpurun_out/ab_masks_c5.log 2>&1; echo c5 rc=$?; cat gpurun_out/ab_masks_c5.log
timeout -k 10 500 bash tools/gpu_variants.sh "--batch 4096 --lmax 10 --dtype f32" plan= ns5=LV_TILE_NSEG=5 ns7=LV_TILE_NSEG=7 plan2= > gpurun_out/ab_nseg_c2.log 2>&1; echo c2 rc=$?; cat gpurun_out/ab_nseg_c2.log
