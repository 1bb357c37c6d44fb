set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/conv_layer_bench_f32.py > gpurun_out/conv_f32.log 2>&1; echo conv rc=$?; cat gpurun_out/conv_f32.log | grep "^{"
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"; grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -1; grep -E "^FAILED|^ERROR" gpurun_out/pytest_gpu.log | head
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.log 2>&1; echo bench rc=$?; grep "^{" gpurun_out/bench_driver.log | cut -c1-600
