# Round-6 same-box A/B experiments (A/B library knobs), one named section per experiment;
# each writes gpurun_out/<name>.log, committed as profiles/r06_<name>.txt.
#   bash tools/gpu_r06_ab.sh <section> ...      e.g. bash tools/gpu_r06_ab.sh nseg slabwt
# Forward sections use tools/gpu_variants.sh (per-variant bench.py + output hashes),
# backward ones tools/bwd_reduce_ab.py (graph-replayed backward alone, dF vs the default).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
AB=$PWD/lie-vae_amd/lie_vae/liblievae_hip_ab.so
C2="--batch 4096 --lmax 10 --dtype f32"
C5="--batch 8192 --lmax 20 --dtype bf16"
fwd() {  # name, bench args, variants...
  local name=$1 args=$2; shift 2
  timeout -k 10 900 bash tools/gpu_variants.sh "$args" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; cat "gpurun_out/$name.log"; return $rc
}
bwd() {  # name, knob list, batches...
  local name=$1 knobs=$2; shift 2
  AB_KNOBS="$knobs" timeout -k 10 600 python -u tools/bwd_reduce_ab.py "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; cat "gpurun_out/$name.log"; return $rc
}
bwd_tests() {  # LV_BWD_VARIANT: the persistent / oracle tests on the A/B library
  LIEVAE_HIP_LIB=$AB LV_BWD_VARIANT=$1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v \
    --timeout 300 --timeout-method thread -k "persistent or shared_spectrum or reproducible or fused_exp_action_bwd" \
    > "gpurun_out/t_bwd_$1.log" 2>&1
  local rc=$?; grep -E "passed|failed" "gpurun_out/t_bwd_$1.log" | tail -2; return $rc
}
for s in "$@"; do
  echo "=== $s"
  case $s in
    # forward, config 2: prologue order (LV_TILE_ANG_ORDER 1 = angles after the spectrum loads)
    ang_order_c2) fwd ab_ang_order_c2 "$C2 --sweep=65536" new=LV_TILE_ANG_ORDER=1 old= new2=LV_TILE_ANG_ORDER=1 old2= ;;
    ang_order_c5) fwd ab_ang_order_c5 "$C5 --sweep=" new=LV_TILE_ANG_ORDER=1 old= new2=LV_TILE_ANG_ORDER=1 old2= ;;
    # forward degree sets: the planner's, degree 0 off the 3-degree wave, LPT on the timeline's
    # per-degree times, pairs summing to 10; then the planner's against the old (cost 40) sets
    masks_c2) fwd ab_masks_c2 "$C2 --sweep=65536" plan= mv0=LV_TILE_MASKS=400:201:102:84:48:30 \
                lpt=LV_TILE_MASKS=400:201:104:12:88:60 pairs=LV_TILE_MASKS=400:202:104:88:50:21 plan2= \
                mv0b=LV_TILE_MASKS=400:201:102:84:48:30 ;;
    masks_c2_planner) fwd ab_masks_c2_planner "$C2 --sweep=65536" plan= old=LV_TILE_MASKS=400:200:102:84:48:31 \
                plan2= old2=LV_TILE_MASKS=400:200:102:84:48:31 ;;
    masks_c5) fwd ab_masks_c5 "$C5 --sweep=" plan= f40=LV_TILE_MASKS=100008:80040:40080:20101:10202:8404:4810:3020 \
                f0=LV_TILE_MASKS=100002:80040:40080:20101:10204:8408:4810:3020 plan2= \
                f40b=LV_TILE_MASKS=100008:80040:40080:20101:10202:8404:4810:3020 ;;
    # forward waves per block across batches, then the planner's rule against the old counts
    nseg_sweep) fwd ab_nseg_sweep "$C2 --sweep=2048,8192,16384,32768,65536" plan= ns4=LV_TILE_NSEG=4 \
                ns5=LV_TILE_NSEG=5 ns6=LV_TILE_NSEG=6 ns7=LV_TILE_NSEG=7 ns8=LV_TILE_NSEG=8 plan2= \
                ns7b=LV_TILE_NSEG=7 ns5b=LV_TILE_NSEG=5 ;;
    nseg_rule) fwd ab_nseg_rule "$C2 --sweep=512,2048,8192,16384,65536" plan= ns6=LV_TILE_NSEG=6 ns4=LV_TILE_NSEG=4 \
                plan2= ns6b=LV_TILE_NSEG=6 ;;
    nseg_c5) fwd ab_nseg_c5 "$C5 --sweep=" plan= ns6=LV_TILE_NSEG=6 ns7=LV_TILE_NSEG=7 ns5=LV_TILE_NSEG=5 plan2= \
                ns7b=LV_TILE_NSEG=7 ;;
    # forward 7-wave degree sets in SIMD-balanced wave order (waves w, w + 4 share a SIMD)
    simd_c2) fwd ab_simd_c2 "$C2 --sweep=512,2048" plan= simd=LV_TILE_MASKS=200:100:81:400:18:42:24 plan2= \
                simd2=LV_TILE_MASKS=200:100:81:400:18:42:24 ;;
    # forward store policy, wave priorities, prologue spread; write-through beyond 24 MB
    fwd_knobs) fwd ab_fwd_knobs "$C2 --sweep=8192,16384" plan= wt0=LV_TILE_WT=0 prio0=LV_TILE_PRIO=0 \
                prio1=LV_TILE_PRIO=1 prio3=LV_TILE_PRIO=3 spread=LV_TILE_SPREAD=1 plan2= ;;
    wt) fwd ab_wt "$C2 --sweep=6144,8192,12288,16384,32768" plan= wt1=LV_TILE_WT=1 plan2= wt1b=LV_TILE_WT=1 ;;
    # backward: degree sets of the persistent kernel's 4 waves
    bwd_masks) bwd ab_bwd_masks "LV_BWD_MASKS=408:211:122:c4,LV_BWD_MASKS=408:211:140:a6,LV_BWD_MASKS=406:211:140:a8,LV_BWD_MASKS=405:240:122:98,LV_BWD_MASKS=410:240:122:8d,LV_BWD_MASKS=408:211:122:c4" 4096 65536 ;;
    # backward: persistent grid of 1 / 2 / 3 blocks per CU at small batches
    bwd_small) bwd ab_bwd_small "LV_BWD_PERSIST_BPC=3,LV_BWD_PERSIST_BPC=1,LV_BWD_PERSIST_BPC=2,LV_BWD_PERSIST_BPC=3,LV_BWD_PERSIST_BPC=2" 4096 8192 ;;
    # backward variants (kBwdVar* bits): 545 round 5, +1024 padded tile, +2048 LDS angle sums;
    # 6689 (+4096 buffer DMA), +8192 lane map, 7713 padded tile by buffer DMA, +16384
    # write-through slab (23073, the product default)
    persist) bwd ab_persist "LV_BWD_VARIANT=545,LV_BWD_VARIANT=1569,LV_BWD_VARIANT=2593,LV_BWD_VARIANT=3617,LV_BWD_VARIANT=545,LV_BWD_VARIANT=3617" 65536 262144 16384 && bwd_tests 3617 ;;
    lanemap) bwd ab_lanemap "LV_BWD_VARIANT=6689,LV_BWD_VARIANT=14881,LV_BWD_VARIANT=6689,LV_BWD_VARIANT=14881" 65536 4096 262144 && bwd_tests 14881 ;;
    padbuf) bwd ab_padbuf "LV_BWD_VARIANT=6689,LV_BWD_VARIANT=7713,LV_BWD_VARIANT=6689,LV_BWD_VARIANT=7713" 65536 262144 4096 16384 && bwd_tests 7713 \
              && LIEVAE_HIP_LIB=$AB LV_BWD_VARIANT=7713 timeout -k 10 600 bash tools/gpu_pmc_bwd_only.sh 65536 action_bwd_persist ;;
    slabwt) bwd ab_slabwt "LV_BWD_VARIANT=6689,LV_BWD_VARIANT=23073,LV_BWD_VARIANT=6689,LV_BWD_VARIANT=23073" 4096 65536 16384 2048 && bwd_tests 23073 ;;
    # fp32 MFMA deconv (LV_DECONV_F32_VARIANT 1 = 128-row tiles, 2 stages; 2 = 3 stages; 3 = 256
    # rows; 4 = 256 rows, 3 stages; 5 = 1 with SIMD-balanced wave tiling, 6 = 3 with it): parity tests and
    # per-layer timing for each (DCF32_VARIANTS overrides the list)
    deconv_f32)
      for v in ${DCF32_VARIANTS:-1 2 3 4 5}; do
        echo "# LV_DECONV_F32_VARIANT=$v" >> gpurun_out/ab_deconv_f32.log
        LIEVAE_HIP_LIB=$AB LV_DECONV_F32_VARIANT=$v timeout -k 10 200 python -u -m pytest tests/test_gpu_configs.py -x -q \
          --timeout 100 --timeout-method thread -k "f32_matches_float64" > gpurun_out/t_dcf32_$v.log 2>&1 || exit 1
        LIEVAE_HIP_LIB=$AB LV_DECONV_F32_VARIANT=$v timeout -k 10 200 python -u tools/deconv_f32_bench.py \
          | grep "^{" >> gpurun_out/ab_deconv_f32.log || exit 1
      done; cat gpurun_out/ab_deconv_f32.log ;;
    # config-3 step eager vs whole-step hipGraph (is the eager bf16 step host-bound?)
    train_graph)
      for cfg in "bf16 --amp bf16 --channels-last" "bf16g --amp bf16 --channels-last --graph" "f32 --amp off" "f32g --amp off --graph"; do
        set -- $cfg; tag=$1; shift
        timeout -k 10 300 python bench_train.py --steps 30 --warmup 10 --no-find "$@" > "gpurun_out/tg_$tag.log" 2>&1 || exit 1
        echo "$tag $(grep '^{' "gpurun_out/tg_$tag.log" | tail -1)" >> gpurun_out/ab_train_graph.log
      done; cat gpurun_out/ab_train_graph.log ;;
    # the train-step record's rounds and host issue time: bench.py twice, bench_train.py alone
    train_diag)
      for i in 1 2; do
        timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "gpurun_out/trd_$i.log" 2>&1 || exit 1
        tail -n 1 "gpurun_out/trd_$i.log" >> gpurun_out/train_diag.log
      done
      timeout -k 10 300 python bench_train.py --steps 30 --warmup 10 --no-find --amp bf16 --channels-last \
        | grep "^{" >> gpurun_out/train_diag.log || exit 1 ;;
    # MIOpen immediate mode (the record's) against find mode (torch caches the picked solver)
    train_find)
      for cfg in "bf16_nofind --amp bf16 --channels-last --no-find" "bf16_find --amp bf16 --channels-last" \
                 "f32_nofind --amp off --no-find" "f32_find --amp off"; do
        set -- $cfg; tag=$1; shift
        timeout -k 10 500 python bench_train.py --steps 30 --warmup 10 "$@" > "gpurun_out/tf_$tag.log" 2>&1 || exit 1
        echo "$tag $(grep '^{' "gpurun_out/tf_$tag.log" | tail -1)" >> gpurun_out/train_find.log
      done; cat gpurun_out/train_find.log ;;
    # in-kernel phase timeline of the config-2 forward (LV_STAMPS)
    timeline) LIEVAE_HIP_LIB=$AB LV_STAMPS=1 timeout -k 10 120 python tools/timeline.py 4096 10 f32 fwd > gpurun_out/timeline_fwd.log 2>&1; cat gpurun_out/timeline_fwd.log ;;
    *) echo "unknown section $s"; exit 2 ;;
  esac || { echo "=== $s failed"; exit 1; }
done
