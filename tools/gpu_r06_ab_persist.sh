# A/B of the persistent backward's round-6 variants (LV_BWD_VARIANT bits, A/B library):
# 545 = product (JIT | single | task1), +1024 padded tile, +2048 LDS angle sums, 3617 both;
# then the persistent / oracle tests on the A/B library with both bits on.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_KNOBS="LV_BWD_VARIANT=545,LV_BWD_VARIANT=1569,LV_BWD_VARIANT=2593,LV_BWD_VARIANT=3617,LV_BWD_VARIANT=545,LV_BWD_VARIANT=3617" \
  timeout -k 10 600 python -u tools/bwd_reduce_ab.py 65536 262144 16384 > gpurun_out/ab_persist.log 2>&1; echo ab rc=$?; cat gpurun_out/ab_persist.log
LIEVAE_HIP_LIB=$PWD/lie-vae_amd/lie_vae/liblievae_hip_ab.so LV_BWD_VARIANT=3617 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread -k "persistent or shared_spectrum or reproducible or fused_exp_action_bwd" > gpurun_out/t_ab.log 2>&1; echo "pytest rc=$?"; grep -E "PASS|FAIL|passed|failed" gpurun_out/t_ab.log | tail -12
