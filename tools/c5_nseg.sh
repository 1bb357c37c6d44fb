#!/bin/bash
# Config-5 forward (l = 20, batch 8192, bf16 out), forced tile segments (LV_TILE_NSEG).
set -u
cd "$(dirname "$0")/.."
export LIEVAE_HIP_LIB="$PWD/lie-vae_amd/lie_vae/liblievae_hip_ab.so"  # the LV_* knobs exist only in the A/B build
for ns in 5 6 7 8; do
  r=$(LV_TILE_NSEG=$ns timeout -k 10 120 python bench.py --lmax 20 --batch 8192 --dtype bf16 --steps 500 --warmup 100 --no-cpu-baseline --cold-launches 0 --no-fwd-bwd --multistream 1 2>/dev/null | grep '^{' | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['roofline']['us_per_launch_events'],3))") || { echo "nseg=$ns failed"; exit 1; }
  echo "l=20 B=8192 bf16 nseg=$ns us=$r"
done
