set -u
mkdir -p gpurun_out
timeout -k 10 120 ./tools/kbench_bwd 4096 300 > gpurun_out/bwd_ab_B4096.txt 2>&1; echo "kbench_bwd rc=$?"; cat gpurun_out/bwd_ab_B4096.txt | head -70
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -k config4 -v -s --timeout 380 --timeout-method thread > gpurun_out/c4.log 2>&1; echo "c4 rc=$?"; grep -E "passed|failed|Error|\[\(1" gpurun_out/c4.log | tail -5
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.log 2>&1 || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/bench_driver.log').read().strip().splitlines()[-1]);print('driver', d['value'], d['roofline']['us_per_launch_events'], d['roofline']['events'], d['roofline']['frac'])"
timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --no-cpu-baseline --cold-launches 0 --no-fwd-bwd > gpurun_out/bench_2000.log 2>&1 || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/bench_2000.log').read().strip().splitlines()[-1]);print('2000', d['value'], d['roofline']['us_per_launch_events'], d['roofline']['events'])"
timeout -k 10 120 ./tools/kbench_fwd 4096 500 > gpurun_out/fwd_ab_B4096.txt 2>&1 || exit 1
head -5 gpurun_out/fwd_ab_B4096.txt
bash tools/gpu_train_prof.sh bf16 bf16_nogemm
