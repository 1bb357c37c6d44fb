set -u
mkdir -p gpurun_out
timeout -k 10 120 ./tools/kbench_bwd 4096 300 > gpurun_out/bwd_ab2_B4096.txt 2>&1; echo "kbench_bwd rc=$?"; head -22 gpurun_out/bwd_ab2_B4096.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 120 python tools/event_probe.py > gpurun_out/event_probe.txt 2>&1; echo "probe rc=$?"; grep -v amdgpu.ids gpurun_out/event_probe.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -k config4 -v -s --timeout 380 --timeout-method thread > gpurun_out/c4.log 2>&1; echo "c4 rc=$?"; grep -E "passed|failed|Error|\[\(1" gpurun_out/c4.log | tail -5
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/trace20 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --cold-launches 0 --no-fwd-bwd --multistream 1 --sweep "" > gpurun_out/trace20.log 2>&1; echo "trace rc=$?"
timeout -k 10 120 ./tools/kbench_fwd 4096 500 > gpurun_out/fwd_ab_B4096.txt 2>&1 || exit 1
head -5 gpurun_out/fwd_ab_B4096.txt
bash tools/gpu_train_prof.sh bf16 bf16_nogemm
