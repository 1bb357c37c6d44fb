#!/bin/bash
# Persistent backward from fewer groups (LV_BWD_PERSIST_MIN) vs the plan's default, backward
# alone at batches below and around the default threshold (769 groups = 4,614 samples).
set -u
cd "$(dirname "$0")/.."
export LIEVAE_HIP_LIB=$PWD/lie-vae_amd/lie_vae/liblievae_hip_ab.so
for r in 1 2; do
for M in 769 1; do
  line="persist_min=$M"
  for B in 1024 2048 4096 6144; do
    out=$(LV_BWD_PERSIST_MIN=$M timeout -k 5 60 python tools/bwd_only.py $B 10 2>/dev/null | tail -1) || exit 1
    line="$line $(echo "$out" | python3 -c 'import json,sys; d=json.load(sys.stdin); print("B%d %.2f" % (d["batch"], d["us_per_call"]))')"
  done
  echo "$line"
done
done
