# Forward tile kernel (config-2 shape, l = 10, C = 10, fp32): wave count per block
# (LV_TILE_NSEG, A/B library) across batch sizes, with the round-6 degree-set cost model.
set -u
mkdir -p gpurun_out
timeout -k 10 900 bash tools/gpu_variants.sh "--batch 4096 --lmax 10 --dtype f32 --sweep=2048,8192,16384,32768,65536" plan= ns4=LV_TILE_NSEG=4 ns5=LV_TILE_NSEG=5 ns6=LV_TILE_NSEG=6 ns7=LV_TILE_NSEG=7 ns8=LV_TILE_NSEG=8 plan2= ns7b=LV_TILE_NSEG=7 ns5b=LV_TILE_NSEG=5 > gpurun_out/ab_nseg_sweep.log 2>&1; echo rc=$?; cat gpurun_out/ab_nseg_sweep.log
