#!/bin/bash
# Backward alone, modular (lv_group_action_bwd) vs fused (lv_fused_exp_action_bwd: + the
# exp -> ZYZ VJP), graph-replayed, same box; then a kernel trace of each at 4,096.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
for r in 1 2; do
for M in modular fused; do
  line="$M"
  for B in 512 4096 16384 65536; do
    out=$(timeout -k 5 60 python tools/bwd_only.py $B 10 $M 2>/dev/null | tail -1) || exit 1
    line="$line $(echo "$out" | python3 -c 'import json,sys; d=json.load(sys.stdin); print("B%d %.2f" % (d["batch"], d["us_per_call"]))')"
  done
  echo "$line"
done
done
for M in modular fused; do
  timeout -k 5 120 rocprofv3 --kernel-trace --stats -d gpurun_out/bwd_$M -o run --output-format csv -- python3 tools/bwd_only.py 4096 20 $M > /dev/null 2>&1 || exit 1
  rm -f gpurun_out/bwd_$M/run_kernel_trace.csv
  echo "== $M 4096"; python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/bwd_$M/run_kernel_stats.csv')): print(r['Calls'], r['AverageNs'], r['MinNs'], r['Name'][:90])"
done
