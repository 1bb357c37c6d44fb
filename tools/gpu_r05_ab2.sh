#!/bin/bash
# Round-5 A/B batch 2: forward with / without the angles output (ang from wave 1 in the
# prologue), persistent backward PMC at 65,536, backward-only kernel trace at 65,536.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
B="--train-steps 0 --config5-launches 0 --no-fwd-bwd --no-cpu-baseline --cold-launches 0 --multistream 1 --steps 400 --warmup 40"
for r in 1 2; do
  for a in "" "--no-ang"; do
    timeout -k 10 120 python bench.py $B $a > gpurun_out/ab2_fwd.json 2>/dev/null || { echo "bench fail"; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab2_fwd.json').read().strip().splitlines()[-1]); print('fwd ang=%s' % ('$a'=='' ), round(d['roofline']['us_per_launch_events'],3), [round(s['us'],1) for s in d['sweep']])"
  done
done
bash tools/gpu_pmc_bwd_only.sh 65536 action_bwd_persist || exit 1
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_bwd_only_65536 -o run --output-format csv -- python3 tools/bwd_only.py 65536 > gpurun_out/r05_bwd_only_65536.json 2>&1 || exit 1
head -4 gpurun_out/r05_bwd_only_65536/run_kernel_stats.csv
