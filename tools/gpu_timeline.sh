#!/bin/bash
# Phase timelines (tools/timeline.py, A/B library with LV_STAMPS=1) at the benchmark shapes.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export LIEVAE_HIP_LIB=$PWD/lie-vae_amd/lie_vae/liblievae_hip_ab.so LV_STAMPS=1
for args in "4096 10 f32 both" "65536 10 f32 fwd" "8192 20 bf16 fwd" "512 10 f32 bwd"; do
  echo "### timeline $args"
  timeout -k 10 120 python tools/timeline.py $args || exit $?
done
