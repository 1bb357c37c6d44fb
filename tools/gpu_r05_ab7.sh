#!/bin/bash
# Persistent backward (one tile buffer): tile wait at the end of the iteration (variant 33)
# vs the first degree's forward recompute ahead of it (41 = 33 | split bit 8); timelines.
set -u
cd "$(dirname "$0")/.."
export LIEVAE_HIP_LIB=$PWD/lie-vae_amd/lie_vae/liblievae_hip_ab.so
for r in 1 2; do
for V in 33 41; do
  for B in 16384 65536 262144; do
    echo "V=$V B=$B $(LV_BWD_VARIANT=$V timeout -k 5 60 python tools/bwd_only.py $B 4 2>/dev/null | tail -1 | python3 -c 'import json,sys; d=json.load(sys.stdin); print("%.2f us gF %s gang %s" % (d["us_per_call"], d["gF_sha"], d["gang_sha"]))')"
  done
done
done
for V in 33 41; do echo "timeline V=$V"; LV_BWD_VARIANT=$V LV_STAMPS=1 timeout -k 5 60 python tools/persist_timeline.py 65536 2>/dev/null; done
