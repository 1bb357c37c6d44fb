#!/bin/bash
# Same-box A/B of the dF slab reduce (LV_BWD_REDUCE = 3 reduce3, 6 reduce5, 7 reduce6),
# backward alone, graph-replayed, at several batches; gF digests per batch must agree.
set -u
cd "$(dirname "$0")/.."
export LIEVAE_HIP_LIB=$PWD/lie-vae_amd/lie_vae/liblievae_hip_ab.so
for r in 1 2; do
for R in 3 6 7; do
  line="reduce=$R"
  for B in 512 4096 16384 65536; do
    out=$(LV_BWD_REDUCE=$R timeout -k 5 60 python tools/bwd_only.py $B 10 2>/dev/null | tail -1) || exit 1
    line="$line $(echo "$out" | python3 -c 'import json,sys; d=json.load(sys.stdin); print("B%d %.2f" % (d["batch"], d["us_per_call"]))')"
  done
  echo "$line"
done
done
