set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -k "mfma_deconv" -q --timeout 200 --timeout-method thread > gpurun_out/deconv_test.log 2>&1; rc=$?; echo "deconv tests rc=$rc"; grep -E "passed|failed|Error|assert|off," gpurun_out/deconv_test.log | head -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/deconv_bwd_bench.py > gpurun_out/deconv_bwd_bench.txt 2>&1; echo "deconv bwd bench rc=$?"; grep -v amdgpu gpurun_out/deconv_bwd_bench.txt
TIMEONLY=1 bash tools/gpu_train_prof.sh bf16_mfma
