#!/bin/bash
# LDS-atomic dF slab (variant bit 256) against the default, one-group (512 / 4,096) and
# persistent (16,384 / 65,536 / 262,144) backward; digests show run-to-run reproducibility.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export LIEVAE_HIP_LIB=$PWD/lie-vae_amd/lie_vae/liblievae_hip_ab.so
for r in 1 2; do
for V in 33 289; do
  for B in 512 4096 16384 65536 262144; do
    echo "V=$V B=$B $(LV_BWD_VARIANT=$V timeout -k 5 60 python tools/bwd_only.py $B 4 2>/dev/null | tail -1 | python3 -c 'import json,sys; d=json.load(sys.stdin); print("%.2f us gF %s gang %s" % (d["us_per_call"], d["gF_sha"], d["gang_sha"]))')"
  done
done
done
python3 - <<'PY'
import numpy as np
for B in (512, 4096, 16384, 65536, 262144):
    a = np.load(f"gpurun_out/bwd_only_gF_{B}_33.npy").astype(np.float64)
    b = np.load(f"gpurun_out/bwd_only_gF_{B}_289.npy").astype(np.float64)
    print(B, "gF rel diff atomic vs default", np.linalg.norm(a - b) / np.linalg.norm(a))
PY
