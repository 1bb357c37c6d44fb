#!/bin/bash
# Same-box A/B of whole library builds, backward alone (graph-replayed) at 4,096 / 65,536 /
# 262,144 samples.  Usage: bash tools/gpu_bwd_libs_ab.sh lib1.so lib2.so ...  (names under
# lie-vae_amd/lie_vae/; "lib.so:V" runs the A/B library with LV_BWD_VARIANT=V)
set -u
cd "$(dirname "$0")/.."
for r in 1 2; do
for spec in "$@"; do
  lib=${spec%%:*}; V=${spec#*:}; [ "$V" = "$spec" ] && V=
  export LIEVAE_HIP_LIB=$PWD/lie-vae_amd/lie_vae/$lib
  line="$spec"
  for B in 4096 65536 262144; do
    us=$(LV_BWD_VARIANT=$V timeout -k 5 60 python tools/bwd_only.py $B 4 2>/dev/null | tail -1 | python3 -c 'import json,sys; d=json.load(sys.stdin); print("%.2f" % d["us_per_call"])') || exit 1
    line="$line bwd$B $us"
  done
  echo "$line"
done
done
