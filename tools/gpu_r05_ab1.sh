#!/bin/bash
# Round-5 A/B batch: persistent-backward tests and batch sweep, forward / backward prologue
# task spreading (A/B library knobs), the default bench line without the train record.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
step() { local name=$1; shift; echo "=== $name $(date +%T)"; "$@"; local rc=$?; echo "=== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step tests timeout -k 10 420 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "persistent or fused_exp_action_bwd_matches or reproducible_and_looped or fused_torch_operator or refuses or fused_vs_oracle or c10_specialised"
step persist_ab bash tools/gpu_bwd_persist_ab.sh
step fwd_spread bash tools/gpu_variants.sh "--sweep 16384,65536" base= spread=LV_TILE_SPREAD=1
step c5_spread bash tools/gpu_variants.sh "--lmax 20 --batch 8192 --dtype bf16 --sweep 65536" base= spread=LV_TILE_SPREAD=1
for V in 1 17; do
  for B in 512 4096; do
    echo "bwd variant $V B=$B $(LIEVAE_HIP_LIB=lie-vae_amd/lie_vae/liblievae_hip_ab.so LV_BWD_VARIANT=$V timeout -k 5 60 python tools/bwd_only.py $B 20 | tail -1 | cut -c1-60)"
  done
done
step bench timeout -k 10 300 python bench.py --train-steps 0 --steps 20 --warmup 5 --cpu-seconds 1
