#!/bin/bash
# MIOpen find-db for the config-3 / config-4 training step's convolutions on MI355X
# (gfx950, 256 CUs): MIOpen's find (torch.backends.cudnn.benchmark) times every solver
# for each conv shape and direction once and records the winners in its user find-db.
# bench.py's train_step record and bench_train.py --no-find then run in immediate mode
# off these records -- without them immediate mode falls back to ConvDirectNaive kernels
# for several NHWC bf16 shapes (30-300 ms per call, profiles/r05_miopen_db_gen.txt).
# Output: lie-vae_amd/lie_vae/data/miopen/*.ufdb.txt, *.udb.txt (text; the compiled-kernel
# cache is not kept).
set -eu
cd "$(dirname "$0")/.."
OUT=gpurun_out/miopen_gen
rm -rf "$OUT" && mkdir -p "$OUT/db" "$OUT/cache"
export MIOPEN_USER_DB_PATH="$PWD/$OUT/db" MIOPEN_CUSTOM_CACHE_DIR="$PWD/$OUT/cache"
for A in "" "--amp bf16 --channels-last"; do
  echo "=== find: bench_train.py $A ($(date +%T))"
  timeout -k 10 600 python bench_train.py --steps 2 --warmup 1 $A
done
mkdir -p lie-vae_amd/lie_vae/data/miopen
cp "$OUT"/db/*.txt gpurun_out/miopen_gen/
ls -la "$OUT/db"
echo "=== done ($(date +%T))"
