#!/bin/bash
# Fused backward at 16,384 / 65,536 (persistent kernel path): the exp -> ZYZ VJP as its own
# launch after the reduce (LV_BWD_VJP_MERGE=0) vs merged with the reduce (1); kernel traces.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp LIEVAE_HIP_LIB=$PWD/lie-vae_amd/lie_vae/liblievae_hip_ab.so
for M in 0 1; do
  for B in 16384 65536; do
    echo "merge=$M $(LV_BWD_VJP_MERGE=$M timeout -k 5 60 python tools/bwd_only.py $B 10 fused 2>/dev/null | tail -1 | python3 -c 'import json,sys; d=json.load(sys.stdin); print("B%d %.2f" % (d["batch"], d["us_per_call"]))')"
  done
  LV_BWD_VJP_MERGE=$M timeout -k 5 120 rocprofv3 --kernel-trace --stats -d gpurun_out/vjpm$M -o run --output-format csv -- python3 tools/bwd_only.py 65536 4 fused > /dev/null 2>&1 || exit 1
  rm -f gpurun_out/vjpm$M/run_kernel_trace.csv
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/vjpm$M/run_kernel_stats.csv')): print('  ', r['Calls'], r['AverageNs'], r['MinNs'], r['Name'][:80])"
done
