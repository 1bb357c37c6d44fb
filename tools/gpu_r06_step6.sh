set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_KNOBS="LV_BWD_VARIANT=2593,LV_BWD_VARIANT=6689,LV_BWD_VARIANT=2593,LV_BWD_VARIANT=6689" timeout -k 10 400 python -u tools/bwd_reduce_ab.py 65536 4096 262144 > gpurun_out/ab_bufdma.log 2>&1; echo ab rc=$?; cat gpurun_out/ab_bufdma.log
LIEVAE_HIP_LIB=$PWD/lie-vae_amd/lie_vae/liblievae_hip_ab.so LV_BWD_VARIANT=6689 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread -k "persistent or shared_spectrum or reproducible or fused_exp_action_bwd" > gpurun_out/t_ab6.log 2>&1; echo "pytest-ab rc=$?"; grep -E "passed|failed" gpurun_out/t_ab6.log | tail -2
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"; grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -1; grep -E "^FAILED|^ERROR|trajectory " gpurun_out/pytest_gpu.log | head
