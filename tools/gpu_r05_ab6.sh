#!/bin/bash
# dF slab reduce: reduce3 (1,024 threads, 8-level tree; default) vs reduce5 (256 threads,
# 12 loads per round, shuffles + one barrier), LV_BWD_REDUCE=3 / 6; digests for determinism.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export LIEVAE_HIP_LIB=$PWD/lie-vae_amd/lie_vae/liblievae_hip_ab.so
for r in 1 2; do
for R in 3 6; do
  for B in 512 4096 65536; do
    echo "R=$R B=$B $(LV_BWD_REDUCE=$R timeout -k 5 60 python tools/bwd_only.py $B 10 2>/dev/null | tail -1 | python3 -c 'import json,sys; d=json.load(sys.stdin); print("%.2f us gF %s" % (d["us_per_call"], d["gF_sha"]))')"
  done
done
done
