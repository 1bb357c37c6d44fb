set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_KNOBS="LV_BWD_VARIANT=6689,LV_BWD_VARIANT=14881,LV_BWD_VARIANT=6689,LV_BWD_VARIANT=14881" timeout -k 10 400 python -u tools/bwd_reduce_ab.py 65536 4096 262144 > gpurun_out/ab_lanemap.log 2>&1; echo ab rc=$?; cat gpurun_out/ab_lanemap.log
LIEVAE_HIP_LIB=$PWD/lie-vae_amd/lie_vae/liblievae_hip_ab.so LV_BWD_VARIANT=14881 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread -k "persistent or shared_spectrum or reproducible or fused_exp_action_bwd" > gpurun_out/t_ab14.log 2>&1; echo "pytest-ab rc=$?"; grep -E "passed|failed" gpurun_out/t_ab14.log | tail -2
