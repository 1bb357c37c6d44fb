#!/bin/bash
# Same-box A/B of whole library builds (LIEVAE_HIP_LIB): backward alone at 4,096 / 65,536,
# forward at 4,096 + sweep, config 5.  Usage: bash tools/gpu_libs_ab.sh lib1.so lib2.so ...
set -u
cd "$(dirname "$0")/.."
B="--train-steps 0 --no-fwd-bwd --no-cpu-baseline --cold-launches 0 --multistream 1 --steps 400 --warmup 40 --config5-launches 200"
for r in 1 2; do
for lib in "$@"; do
  export LIEVAE_HIP_LIB=$PWD/lie-vae_amd/lie_vae/$lib
  b1=$(timeout -k 5 60 python tools/bwd_only.py 4096 20 | tail -1 | python3 -c 'import json,sys; print("%.2f" % json.load(sys.stdin)["us_per_call"])') || exit 1
  b2=$(timeout -k 5 60 python tools/bwd_only.py 65536 4 | tail -1 | python3 -c 'import json,sys; print("%.1f" % json.load(sys.stdin)["us_per_call"])') || exit 1
  f=$(timeout -k 10 120 python bench.py $B 2>/dev/null | tail -1 | python3 -c 'import json,sys; d=json.load(sys.stdin); print("fwd %.2f sweep %s c5 %.1f" % (d["roofline"]["us_per_launch_events"], [round(s["us"],1) for s in d["sweep"]], d["config5"]["us_per_launch"]))') || exit 1
  echo "$lib bwd4096 $b1 bwd65536 $b2 $f"
done
done
