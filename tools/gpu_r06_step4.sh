set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bf16_trajectory.py 50 s2s2 1 > gpurun_out/traj_nd.log 2>&1; echo traj rc=$?; grep -E "step (0|45)|^(f32_pert|bf16)" gpurun_out/traj_nd.log
AB_KNOBS="LV_BWD_PERSIST_MIN=0,LV_BWD_PERSIST_MIN=1,LV_BWD_PERSIST_MIN=0,LV_BWD_PERSIST_MIN=1" timeout -k 10 300 python -u tools/bwd_reduce_ab.py 4096 2048 > gpurun_out/ab_persist_small.log 2>&1; echo ab rc=$?; cat gpurun_out/ab_persist_small.log
timeout -k 10 400 bash tools/gpu_pmc_bwd_only.sh 65536 action_bwd_persist > gpurun_out/pmc65536.log 2>&1; echo pmc rc=$?; head -20 gpurun_out/pmc65536.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"; grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -1; grep -E "^FAILED|^ERROR|trajectory " gpurun_out/pytest_gpu.log | head
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.log 2>&1; echo bench rc=$?
