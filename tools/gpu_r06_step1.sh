set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread -k "shared_spectrum" > gpurun_out/t1.log 2>&1; echo "pytest rc=$?"; tail -5 gpurun_out/t1.log
timeout -k 10 500 python -u tools/bf16_trajectory.py 50 s2s2 > gpurun_out/traj_s2s2.log 2>&1; echo traj rc=$?; tail -3 gpurun_out/traj_s2s2.log
timeout -k 10 300 python -u tools/bf16_trajectory.py 50 alg > gpurun_out/traj_alg.log 2>&1; echo traj2 rc=$?; tail -3 gpurun_out/traj_alg.log
timeout -k 10 400 bash tools/gpu_pmc_bwd_only.sh 4096 action_bwd_tile > gpurun_out/pmc4096.log 2>&1; echo pmc rc=$?; tail -40 gpurun_out/pmc4096.log
