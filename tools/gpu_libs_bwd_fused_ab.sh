#!/bin/bash
# Same-box A/B of library builds: backward alone, modular and fused, at 512 / 4,096 /
# 65,536 samples.  Usage: bash tools/gpu_libs_bwd_fused_ab.sh lib1.so lib2.so ...
set -u
cd "$(dirname "$0")/.."
for r in 1 2; do
for lib in "$@"; do
  export LIEVAE_HIP_LIB=$PWD/lie-vae_amd/lie_vae/$lib
  line="$lib"
  for M in modular fused; do
    for B in 512 4096 65536; do
      out=$(timeout -k 5 60 python tools/bwd_only.py $B 10 $M 2>/dev/null | tail -1) || exit 1
      line="$line $(echo "$out" | python3 -c 'import json,sys; d=json.load(sys.stdin); print("%s%d %.2f" % ("f" if d["fused"] else "m", d["batch"], d["us_per_call"]))')"
    done
  done
  echo "$line"
done
done
