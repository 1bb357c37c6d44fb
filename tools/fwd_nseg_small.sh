#!/bin/bash
# Forward tile kernel, forced segment counts (LV_TILE_NSEG) at small batches: HIP-event
# us per launch of the config-2 fused forward (l = 10, C = 10, fp32).
set -u
cd "$(dirname "$0")/.."
export LIEVAE_HIP_LIB="$PWD/lie-vae_amd/lie_vae/liblievae_hip_ab.so"  # the LV_* knobs exist only in the A/B build
mkdir -p gpurun_out
for B in 512 2048 4096; do
  for ns in 4 6 8; do
    r=$(LV_TILE_NSEG=$ns timeout -k 10 120 python bench.py --batch $B --steps 2000 --warmup 200 --no-cpu-baseline --cold-launches 0 --no-fwd-bwd --multistream 1 2>/dev/null | grep '^{' | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['roofline']['us_per_launch_events'],3))") || { echo "B=$B nseg=$ns failed"; exit 1; }
    echo "B=$B nseg=$ns us=$r"
  done
done
