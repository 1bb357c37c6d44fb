#!/bin/bash
# Persistent backward variants after the no-SLP / literal-multiply build: default (1),
# single tile buffer at 3 blocks per CU (33), non-JIT chain (65), 5 waves per block (129).
set -u
cd "$(dirname "$0")/.."
for r in 1 2; do
for V in 1 33 65 129 161; do
  for B in 32768 65536 262144; do
    echo "persist variant $V B=$B $(LIEVAE_HIP_LIB=$PWD/lie-vae_amd/lie_vae/liblievae_hip_ab.so LV_BWD_VARIANT=$V timeout -k 5 60 python tools/bwd_only.py $B 4 2>/dev/null | tail -1 | cut -c1-70)"
  done
done
done
