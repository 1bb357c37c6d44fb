set -u
mkdir -p gpurun_out
timeout -k 10 120 ./tools/kbench_fwd 4096 1000 > gpurun_out/fwd_mreg_B4096.txt 2>&1; echo "fwd4096 rc=$?"; cat gpurun_out/fwd_mreg_B4096.txt
timeout -k 10 120 ./tools/kbench_fwd 65536 200 > gpurun_out/fwd_mreg_B65536.txt 2>&1; echo "fwd65536 rc=$?"; tail -5 gpurun_out/fwd_mreg_B65536.txt
timeout -k 10 200 ./tools/kbench_c5 8192 200 mreg > gpurun_out/c5_mreg.txt 2>&1; echo "c5 rc=$?"; cat gpurun_out/c5_mreg.txt
TIMEONLY=1 bash tools/gpu_train_prof.sh bf16_phase f32_nbn f32_phase
