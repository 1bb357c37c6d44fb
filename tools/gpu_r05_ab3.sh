#!/bin/bash
# Round-5 A/B batch 3: library builds (SLP off, J rows' first term as a multiply) and the
# persistent backward's variants (single tile buffer at 3 blocks per CU, non-JIT chain).
set -u
cd "$(dirname "$0")/.."
bash tools/gpu_libs_ab.sh liblievae_hip.so liblievae_hip_xnoslp.so liblievae_hip_xjmm.so liblievae_hip_xboth.so || exit 1
for V in 1 33 65 97; do
  for B in 32768 65536; do
    echo "persist variant $V B=$B $(LIEVAE_HIP_LIB=$PWD/lie-vae_amd/lie_vae/liblievae_hip_ab.so LV_BWD_VARIANT=$V timeout -k 5 60 python tools/bwd_only.py $B 4 | tail -1 | cut -c1-70)"
  done
done
