#!/bin/bash
# A/B of the bf16 tile-kernel options at config 5 (l = 20, B = 8192, bf16 out) with the A/B
# library: LV_TILE_BF16 option bits (1 pair-row writes, 4 spectrum in the tile's last two
# slots) x LV_TILE_SW samples per block.  Per variant: the output fingerprint (must match
# the base bit for bit) and bench.py's per-launch time (+ the 65,536 sweep point).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/c5_knobs
mkdir -p $OUT
export LIEVAE_HIP_LIB=$PWD/lie-vae_amd/lie_vae/liblievae_hip_ab.so
for v in "0 6" "1 6" "4 6" "5 6" "4 5" "5 5" "0 6"; do
  set -- $v
  tag="f$1_sw$2"
  LV_TILE_BF16=$1 LV_TILE_SW=$2 timeout -k 10 120 python tools/c5_hash.py > $OUT/$tag.hash 2>&1 || { echo "$tag hash failed"; tail -3 $OUT/$tag.hash; exit 1; }
  LV_TILE_BF16=$1 LV_TILE_SW=$2 timeout -k 10 240 python bench.py --lmax 20 --batch 8192 --dtype bf16 --steps 400 --warmup 40 \
      --no-fwd-bwd --no-cpu-baseline --cold-launches 0 --multistream 1 --sweep 65536 > $OUT/$tag.log 2>&1 || { echo "$tag bench failed"; tail -3 $OUT/$tag.log; exit 1; }
  python3 - "$tag" $OUT/$tag.log $OUT/$tag.hash <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[2]) if l.startswith("{")][-1]
h = [l for l in open(sys.argv[3]) if l.startswith("{")][-1].strip()
r = d["roofline"]
sw = " ".join(f'{s["batch"]}:{s["us"]:.1f}us' for s in d.get("sweep") or [])
print(f'{sys.argv[1]:>10}  B8192 {r["us_per_launch_events"]:6.2f} us (raw {r["us_per_launch_events_raw"]:6.2f})  {sw}  {h}')
PY
done
echo done
