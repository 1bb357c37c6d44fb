#!/bin/bash
# Fused backward on the one-group kernel (below 769 groups): the exp -> ZYZ VJP in the tile
# kernel's tail (LV_BWD_TAIL_VJP=1) vs beside the dF reduce in its launch (0); same box.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp LIEVAE_HIP_LIB=$PWD/lie-vae_amd/lie_vae/liblievae_hip_ab.so
for r in 1 2; do
for T in 1 0; do
  line="tail_vjp=$T"
  for B in 512 1024 2048 4096; do
    out=$(LV_BWD_TAIL_VJP=$T timeout -k 5 60 python tools/bwd_only.py $B 10 fused 2>/dev/null | tail -1) || exit 1
    line="$line $(echo "$out" | python3 -c 'import json,sys; d=json.load(sys.stdin); print("B%d %.2f %s" % (d["batch"], d["us_per_call"], d["gF_sha"]))')"
  done
  echo "$line"
done
done
