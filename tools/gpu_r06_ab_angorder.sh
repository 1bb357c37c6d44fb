# A/B of the forward prologue order (LV_TILE_ANG_ORDER: 1 = angles after the spectrum loads
# are issued, the new default; 0 = round 5), config 2 (+ sweep) and config 5, then the
# phase timeline at config 2.
set -u
mkdir -p gpurun_out
timeout -k 10 500 bash tools/gpu_variants.sh "--batch 4096 --lmax 10 --dtype f32 --sweep=65536" new= old=LV_TILE_ANG_ORDER=0 new2= old2=LV_TILE_ANG_ORDER=0 > gpurun_out/ab_ang_c2.log 2>&1; echo c2 rc=$?; cat gpurun_out/ab_ang_c2.log
timeout -k 10 500 bash tools/gpu_variants.sh "--batch 8192 --lmax 20 --dtype bf16 --sweep=" new= old=LV_TILE_ANG_ORDER=0 new2= old2=LV_TILE_ANG_ORDER=0 > gpurun_out/ab_ang_c5.log 2>&1; echo c5 rc=$?; cat gpurun_out/ab_ang_c5.log
LIEVAE_HIP_LIB=$PWD/lie-vae_amd/lie_vae/liblievae_hip_ab.so LV_STAMPS=1 timeout -k 10 120 python tools/timeline.py 4096 10 f32 fwd > gpurun_out/tl_fwd2.txt 2>&1; echo tl rc=$?; grep -v amdgpu.ids gpurun_out/tl_fwd2.txt
# degree sets of the config-2 forward (LV_TILE_MASKS, one hex mask per wave): the planner's
# cost-balanced sets, degree 0 moved off the 3-degree wave, LPT over the timeline's per-degree
# times, pairs summing to 10
timeout -k 10 600 bash tools/gpu_variants.sh "--batch 4096 --lmax 10 --dtype f32 --sweep=" plan= mv0=LV_TILE_MASKS=400,201,102,84,48,30 lpt=LV_TILE_MASKS=400,201,104,12,88,60 pairs=LV_TILE_MASKS=400,202,104,88,50,21 plan2= mv0b=LV_TILE_MASKS=400,201,102,84,48,30 > gpurun_out/ab_masks_c2.log 2>&1; echo masks rc=$?; cat gpurun_out/ab_masks_c2.log
