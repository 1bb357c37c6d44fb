set -u
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.log 2>&1 || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/bench_driver.log').read().strip().splitlines()[-1]);r=d['roofline'];print('driver', d['value'], r['us_per_launch_events'], r['us_per_launch_events_raw'], r['us_one_launch_bracket'], r['frac'])"
TIMEONLY=1 bash tools/gpu_train_prof.sh bf16 bf16_nbn bf16_gemv bf16_both f32_both
