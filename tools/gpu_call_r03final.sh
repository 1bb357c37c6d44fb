# Round-3 final HEAD check: full GPU suite, smoke, driver-form bench
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -v -rf --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -1 gpurun_out/pytest_gpu.log; grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_driver.log | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; fb=d['fwd_bwd']
print('c2 us', round(r['us_per_launch_events'],3), 'frac', round(r['frac'],4), 'value', round(d['value']/1e6,1), 'M/s')
print('fwd+bwd us', round(fb['us_per_step'],2), 'bwd us', round(fb['action_bwd']['us_per_call'],2), 'sweep', [(s['batch'], round(s['us'],1), round(s['frac'],3)) for s in d['sweep']])"
