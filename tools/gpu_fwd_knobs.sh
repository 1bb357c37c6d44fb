#!/bin/bash
# A/B of the metric forward tile kernel's launch shape (A/B library knobs): flush store
# policy (LV_TILE_WT: 0 nt,
# 1 sc1 write-through, 2 plain).  Per variant: bench.py's B = 4096 events figure and the
# 16K / 65K / 262K sweep.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/fwd_knobs
export LIEVAE_HIP_LIB=$PWD/lie-vae_amd/lie_vae/liblievae_hip_ab.so
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 240 python bench.py --steps 400 --warmup 50 --no-fwd-bwd --no-cpu-baseline \
      --cold-launches 0 --sweep 16384,65536,262144 > gpurun_out/fwd_knobs/$tag.log 2>&1 || { echo "$tag failed"; tail -3 gpurun_out/fwd_knobs/$tag.log; exit 1; }
  python3 - "$tag" gpurun_out/fwd_knobs/$tag.log <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[2]) if l.startswith("{")][-1]
sw = " ".join(f'{r["batch"]}:{r["us"]:.2f}us/{r["frac"]:.3f}' for r in d.get("sweep", []))
print(f'{sys.argv[1]:>14}  B4096 {d.get("us_per_launch_events", 0):6.2f} us  {sw}')
PY
}
run base
run prio0 LV_TILE_PRIO=0
run prio3 LV_TILE_PRIO=3
run base2
# config 5 (l = 20, B = 8192, bf16 out): one-shot tile kernel vs the persistent one
run_c5() {
  local tag=$1; shift
  env "$@" timeout -k 10 240 python bench.py --lmax 20 --batch 8192 --dtype bf16 --steps 300 --warmup 30 --no-fwd-bwd \
      --no-cpu-baseline --cold-launches 0 --multistream 1 --sweep 65536 > gpurun_out/fwd_knobs/$tag.log 2>&1 || { echo "$tag failed"; tail -3 gpurun_out/fwd_knobs/$tag.log; exit 1; }
  python3 - "$tag" gpurun_out/fwd_knobs/$tag.log <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[2]) if l.startswith("{")][-1]
sw = " ".join(f'{r["batch"]}:{r["us"]:.2f}us/{r["frac"]:.3f}' for r in d.get("sweep", []))
print(f'{sys.argv[1]:>14}  B8192 {d.get("us_per_launch_events", 0):6.2f} us  {sw}')
PY
}
run_c5 c5base
run_c5 c5prio0 LV_TILE_PRIO=0
run_c5 c5base2
