set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -k "fused_bn or mfma_deconv_backward" -q --timeout 200 --timeout-method thread > gpurun_out/bn_test.log 2>&1; rc=$?; echo "bn tests rc=$rc"; grep -E "passed|failed|Error|assert|off," gpurun_out/bn_test.log | head -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bn_bench.py > gpurun_out/bn_bench.txt 2>&1; echo "bn bench rc=$?"; grep -v amdgpu gpurun_out/bn_bench.txt
TIMEONLY=1 bash tools/gpu_train_prof.sh bf16_mfma
