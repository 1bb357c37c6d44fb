# bench.py twice (driver form) and bench_train.py alone: the train-step rounds with the host issue time per step
set -u
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/trd_$i.log 2>&1 || { tail -5 gpurun_out/trd_$i.log; exit 1; }
tail -n 1 gpurun_out/trd_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); t=d['train_step']; [print(k, [round(x,2) for x in t[k]['ms_per_step_rounds']], [round(x,2) for x in t[k]['host_issue_ms_per_step_rounds']]) for k in ('bf16','f32')]"
done
timeout -k 10 300 python bench_train.py --steps 30 --warmup 10 --no-find --amp bf16 --channels-last > gpurun_out/trd_bt.log 2>&1 || exit 1
grep "^{" gpurun_out/trd_bt.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('standalone', round(d['ms_per_step'],2), [round(x,2) for x in d['host_issue_ms_per_step_rounds']])"
