set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread -k "f32 or config3_conv_vae or graph_replay or trajectory or dp_trainer" > gpurun_out/chk_f32.log 2>&1; rc=$?
grep -E "PASS|FAIL|passed|failed" gpurun_out/chk_f32.log | tail -16; exit $rc
