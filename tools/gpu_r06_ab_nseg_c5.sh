# Config-5 forward (l = 20, bf16 out, B = 8,192): waves per block (LV_TILE_NSEG, A/B library)
# with the round-6 degree-set cost model.
set -u
mkdir -p gpurun_out
timeout -k 10 800 bash tools/gpu_variants.sh "--batch 8192 --lmax 20 --dtype bf16 --sweep=" plan= ns6=LV_TILE_NSEG=6 ns7=LV_TILE_NSEG=7 ns5=LV_TILE_NSEG=5 plan2= ns7b=LV_TILE_NSEG=7 > gpurun_out/ab_nseg_c5.log 2>&1; echo rc=$?; cat gpurun_out/ab_nseg_c5.log
