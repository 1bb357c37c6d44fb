set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "wave_counts or other_grid_sizes" > gpurun_out/newtests.log 2>&1; rc=$?
grep -E "PASS|FAIL|passed|failed|Error" gpurun_out/newtests.log | tail -8; exit $rc
