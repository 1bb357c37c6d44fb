# Round-3 final evidence at HEAD: driver-form bench line, config-2-only rocprof, config 5
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_driver.log | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; fb=d['fwd_bwd']
print('c2 us', round(r['us_per_launch_events'],3), 'frac', round(r['frac'],4), 'traffic', r['traffic'], 'value', round(d['value']/1e6,1), 'M/s', 'cpu', d['cpu_baseline']['value'])
print('fwd+bwd us', round(fb['us_per_step'],2), 'bwd us', round(fb['action_bwd']['us_per_call'],2), 'sweep', [(s['batch'], round(s['us'],1), round(s['frac'],3)) for s in d['sweep']])"
rm -rf gpurun_out/prof_c2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- python3 bench.py --steps 2000 --warmup 200 --no-cpu-baseline --multistream 1 --cold-launches 0 --no-fwd-bwd --sweep "" > gpurun_out/prof_c2.log 2>&1 || exit $?
find gpurun_out/prof_c2 -name "*kernel_trace.csv" -delete
timeout -k 10 300 python bench.py --lmax 20 --batch 8192 --dtype bf16 --no-cpu-baseline --steps 500 --sweep 65536 > gpurun_out/bench_c5.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_c5.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 us', round(d['roofline']['us_per_launch_events'],2), round(d['roofline']['frac'],3))"
