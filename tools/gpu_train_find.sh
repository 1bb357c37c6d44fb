# config-3 bf16 / fp32 step: MIOpen immediate mode (--no-find, the bench record's mode) against
# find mode (cudnn.benchmark: torch caches the picked solver per shape), rounds + host issue time.
set -u
mkdir -p gpurun_out
for cfg in "bf16_nofind --amp bf16 --channels-last --no-find" "bf16_find --amp bf16 --channels-last" "f32_nofind --amp off --no-find" "f32_find --amp off"; do
  set -- $cfg; tag=$1; shift
  timeout -k 10 500 python bench_train.py --steps 30 --warmup 10 "$@" > gpurun_out/tf_$tag.log 2>&1 || { echo "$tag failed"; tail -5 gpurun_out/tf_$tag.log; exit 1; }
  echo "$tag $(grep '^{' gpurun_out/tf_$tag.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), [round(x,2) for x in d["host_issue_ms_per_step_rounds"]], round(d["warmup_s"],1))')"
done
