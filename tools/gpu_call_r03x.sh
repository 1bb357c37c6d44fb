# HEAD evidence: full GPU suite, smoke, driver-form bench, dF reduce A/B, config-3 step timing
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -v -rf --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -1 gpurun_out/pytest_gpu.log; grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.log 2>&1 || { echo bench failed; tail gpurun_out/bench_driver.log; exit 1; }
grep '^{' gpurun_out/bench_driver.log | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; fb=d['fwd_bwd']
print('c2 us', round(r['us_per_launch_events'],3), 'frac', round(r['frac'],4), 'traffic', r['traffic'], 'value', round(d['value']/1e6,1), 'M/s')
print('fwd+bwd us', round(fb['us_per_step'],2), 'bwd us', round(fb['action_bwd']['us_per_call'],2), 'sweep', [(s['batch'], round(s['us'],1), round(s['frac'],3)) for s in d['sweep']])"
timeout -k 10 400 python tools/bwd_reduce_ab.py 4096 512 > gpurun_out/bwd_reduce_ab2.txt 2>&1; cat gpurun_out/bwd_reduce_ab2.txt
timeout -k 10 300 python bench_train.py --steps 30 --warmup 5 --amp bf16 --channels-last > gpurun_out/train_c3.log 2>&1 && grep '^{' gpurun_out/train_c3.log | tail -1 | cut -c1-200
