# fp32 MFMA transposed convolution: parity tests, then the per-layer timing against MIOpen.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 200 --timeout-method thread -k "f32_matches_float64 or f32_module" > gpurun_out/deconv_f32_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|error|passed|failed" gpurun_out/deconv_f32_tests.log | tail -15
[ $rc -eq 0 ] || { tail -40 gpurun_out/deconv_f32_tests.log; exit $rc; }
timeout -k 10 300 python -u tools/deconv_f32_bench.py > gpurun_out/deconv_f32_bench.log 2>&1; echo bench rc=$?; cat gpurun_out/deconv_f32_bench.log | tail -5
