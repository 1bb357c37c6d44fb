set -u
mkdir -p gpurun_out/trainprof2
export TMPDIR=/tmp
B="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-fwd-bwd --sweep= --config5-launches 0 --multistream 0 --cold-launches 0"
timeout -k 10 300 $B > gpurun_out/bt1.log 2>&1; echo a rc=$?; grep '^{' gpurun_out/bt1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k:v['ms_per_step'] for k,v in d['train_step'].items() if isinstance(v,dict)})"
timeout -k 10 300 $B --train-warmup 10 --train-steps 20 > gpurun_out/bt2.log 2>&1; echo b rc=$?; grep '^{' gpurun_out/bt2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k:v['ms_per_step'] for k,v in d['train_step'].items() if isinstance(v,dict)})"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/trainprof2 -o run --output-format csv -- $B > gpurun_out/bt_prof.log 2>&1; echo prof rc=$?
find gpurun_out/trainprof2 -name "*kernel_trace.csv" -delete
