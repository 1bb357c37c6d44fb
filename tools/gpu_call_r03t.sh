# deconv v2 default + fused decoder ReLU: GPU tests, layer bench, config-3 step A/B
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py -k "deconv or relu or config3 or fused_bn" -v --timeout 240 --timeout-method thread > gpurun_out/deconv_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/deconv_tests.log | sed 's/tests\/test_gpu_configs.py:://' | head -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/deconv_bench.py > gpurun_out/deconv_v2.txt 2>&1 || exit $?
TIMEONLY=1 bash tools/gpu_train_prof.sh bf16_mfma bf16_norelu bf16_mfma
