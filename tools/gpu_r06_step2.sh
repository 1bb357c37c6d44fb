set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/bf16_trajectory.py 50 s2s2 0,1,2 > gpurun_out/traj_heads.log 2>&1; echo traj rc=$?; grep -E "^(f32_pert|bf16)" gpurun_out/traj_heads.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -v --timeout 300 --timeout-method thread -k "bf16_step_matches" > gpurun_out/t2.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/t2.log; cat gpurun_out/bf16_step_report.json
