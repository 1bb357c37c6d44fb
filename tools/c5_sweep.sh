#!/bin/bash
# Config 5 (l = 20, batch 8192, bf16 out): tile kernel vs the segment-grid kernel at
# several segment counts (LV_FWD_NSEG, A/B only).  One bench process per point.
cd "$(dirname "$0")/.."
export LIEVAE_HIP_LIB="$PWD/lie-vae_amd/lie_vae/liblievae_hip_ab.so"  # the LV_* knobs exist only in the A/B build
run() { timeout -k 10 120 env "$@" python bench.py --no-cpu-baseline --lmax 20 --batch 8192 --dtype bf16 --steps 400 --warmup 50 --cold-launches 0 --multistream 1 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$*', round(d['roofline']['us_per_launch_events'],2), 'us', round(d['roofline']['frac'],3))"; }
run LV_TILE=1
for ns in 2 4 6 8 12 16; do run LV_TILE=0 LV_FWD_NSEG=$ns; done
