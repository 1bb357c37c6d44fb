# Forward tile kernel store policy beyond the write-through threshold (24 MB of output):
# LV_TILE_WT=1 forces write-through (sc1) stores at every size, 0 nt everywhere.
set -u
mkdir -p gpurun_out
timeout -k 10 600 bash tools/gpu_variants.sh "--batch 4096 --lmax 10 --dtype f32 --sweep=6144,8192,12288,16384,32768" plan= wt1=LV_TILE_WT=1 plan2= wt1b=LV_TILE_WT=1 > gpurun_out/ab_wt.log 2>&1; echo rc=$?; cat gpurun_out/ab_wt.log
