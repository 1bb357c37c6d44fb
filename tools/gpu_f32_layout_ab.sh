#!/bin/bash
# fp32 config-3 training step, NCHW vs channels-last, MIOpen find mode (every solver timed
# once per shape), same box.
set -u
cd "$(dirname "$0")/.."
export MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_f32/db MIOPEN_CUSTOM_CACHE_DIR=$PWD/gpurun_out/miopen_f32/cache
mkdir -p $MIOPEN_USER_DB_PATH $MIOPEN_CUSTOM_CACHE_DIR
for A in "" "--channels-last"; do
  echo "=== fp32 $A ($(date +%T))"
  timeout -k 10 500 python bench_train.py --steps 10 --warmup 3 $A 2>&1 | tail -2 || exit 1
done
for A in "" "--channels-last"; do
  echo "=== fp32 rerun (db warm) $A ($(date +%T))"
  timeout -k 10 300 python bench_train.py --steps 10 --warmup 3 $A 2>&1 | tail -1 || exit 1
done
