# Two bench.py runs (default, then the driver's form): the train-step records' round spread.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/b_tr.log 2>&1 || { tail -5 gpurun_out/b_tr.log; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/b_tr2.log 2>&1 || { tail -5 gpurun_out/b_tr2.log; exit 1; }
for f in gpurun_out/b_tr.log gpurun_out/b_tr2.log; do
  tail -n 1 $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); t=d['train_step']; print(d['value'], t['bf16']['ms_per_step_rounds'], t['f32']['ms_per_step_rounds'])"
done
