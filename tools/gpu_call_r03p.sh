# Degree-split tile kernel: bitwise test, then the launch-shape A/B (config 2 + sweep, config 5).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "degree_split or tile_kernel or group_action" -v --timeout 300 --timeout-method thread > gpurun_out/split_test.log 2>&1; rc=$?
echo "split tests rc=$rc"; grep -E "PASSED|FAILED|Error|assert" gpurun_out/split_test.log | head -30
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_fwd_knobs.sh
