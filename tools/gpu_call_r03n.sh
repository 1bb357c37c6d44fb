set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "persistent_wave or global_spectrum" -q --timeout 200 --timeout-method thread > gpurun_out/ws_test.log 2>&1; rc=$?; echo "ws tests rc=$rc"; grep -E "passed|failed|Error|assert" gpurun_out/ws_test.log | head -12
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_fwd_knobs.sh
