#!/bin/bash
# A/B of A/B-library knob settings on one bench.py shape, each variant also fingerprinted
# (tools/c5_hash.py: must match the first variant bit for bit where the arithmetic is the
# same).  Usage:
#   bash tools/gpu_variants.sh "<bench.py args>" tag=VAR=val,VAR=val tag2=... 
# e.g. bash tools/gpu_variants.sh "--lmax 20 --batch 8192 --dtype bf16" base= sw5=LV_TILE_SW=5
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/variants
mkdir -p $OUT
export LIEVAE_HIP_LIB=$PWD/lie-vae_amd/lie_vae/liblievae_hip_ab.so
BARGS=$1; shift
for spec in "$@"; do
  tag=${spec%%=*}; envs=${spec#*=}
  IFS=',' read -ra kv <<< "$envs"
  timeout -k 10 120 env ${kv[@]+"${kv[@]}"} python tools/c5_hash.py > $OUT/$tag.hash 2>&1 || { echo "$tag hash failed"; tail -3 $OUT/$tag.hash; exit 1; }
  timeout -k 10 300 env ${kv[@]+"${kv[@]}"} python bench.py $BARGS --steps 400 --warmup 40 --no-fwd-bwd --no-cpu-baseline \
      --cold-launches 0 --multistream 1 --config5-launches 0 --train-steps 0 > $OUT/$tag.log 2>&1 || { echo "$tag bench failed"; tail -3 $OUT/$tag.log; exit 1; }
  python3 - "$tag" $OUT/$tag.log $OUT/$tag.hash <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[2]) if l.startswith("{")][-1]
h = [l for l in open(sys.argv[3]) if l.startswith("{")][-1].strip()
r = d["roofline"]
sw = " ".join(f'{s["batch"]}:{s["us"]:.1f}' for s in d.get("sweep") or [])
print(f'{sys.argv[1]:>10} {r["us_per_launch_events"]:7.2f} us  sweep {sw}  {h}', flush=True)
PY
done
