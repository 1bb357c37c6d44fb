# fp32 MFMA deconv forward in the fp32 training step: the config tests (fp32 VAE parity,
# the fp32 MFMA layer tests, the trajectories), the per-layer timing and the bench line.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread > gpurun_out/f32step_tests.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/f32step_tests.log | tail -3
[ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/f32step_tests.log | head; tail -30 gpurun_out/f32step_tests.log; exit $rc; }
timeout -k 10 200 python -u tools/deconv_f32_bench.py > gpurun_out/f32step_layers.log 2>&1 || { tail -5 gpurun_out/f32step_layers.log; exit 1; }
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/f32step_bench.log 2>&1 || { tail -5 gpurun_out/f32step_bench.log; exit 1; }
tail -n 1 gpurun_out/f32step_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('us', d['roofline']['us_per_launch_events'], 'train', {k: (d['train_step'][k]['ms_per_step'], d['train_step'][k]['ms_per_step_rounds']) for k in ('f32','bf16')})"
