set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_KNOBS="LV_BWD_VARIANT=545,LV_BWD_VARIANT=2593,LV_BWD_VARIANT=545,LV_BWD_VARIANT=2593" timeout -k 10 300 python -u tools/bwd_reduce_ab.py 65536 > gpurun_out/ab_ang2.log 2>&1; echo ab rc=$?; cat gpurun_out/ab_ang2.log
AB_KNOBS="LV_BWD_PERSIST_MIN=0,LV_BWD_PERSIST_MIN=1,LV_BWD_PERSIST_MIN=1+LV_BWD_PERSIST_BPC=2,LV_BWD_PERSIST_MIN=1+LV_BWD_PERSIST_BPC=1,LV_BWD_PERSIST_MIN=0,LV_BWD_PERSIST_MIN=1" timeout -k 10 500 python -u tools/bwd_reduce_ab.py 4096 1024 512 > gpurun_out/ab_small.log 2>&1; echo ab rc=$?; cat gpurun_out/ab_small.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -v -s -rf --timeout 300 --timeout-method thread -k "trajectory or persistent or shared_spectrum or fused_exp_action_bwd" > gpurun_out/t5.log 2>&1; echo "pytest rc=$?"; grep -E "passed|failed|trajectory |PASS|FAIL" gpurun_out/t5.log | tail -12
cat gpurun_out/bf16_trajectory_report.json | head -40
