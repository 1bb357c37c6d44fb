# config-3 training step, eager vs whole-step hipGraph (DPTrainer graph=True), bf16 and fp32,
# each in its own process, twice: is the eager bf16 step host-bound on this box?
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
for cfg in "bf16 --amp bf16 --channels-last" "bf16g --amp bf16 --channels-last --graph" "f32 --amp off" "f32g --amp off --graph"; do
  set -- $cfg; tag=$1; shift
  timeout -k 10 300 python bench_train.py --steps 30 --warmup 10 --no-find "$@" > gpurun_out/tg_${tag}_$rep.log 2>&1 || { echo "$tag failed"; tail -5 gpurun_out/tg_${tag}_$rep.log; exit 1; }
  echo "$tag rep$rep: $(grep '^{' gpurun_out/tg_${tag}_$rep.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), d.get("config",{}).get("launch"))')"
done
done
