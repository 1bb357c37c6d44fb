# deconv v2 default + fused decoder ReLU: GPU tests, layer bench, config-3 step A/B
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py -k "deconv or relu or config3 or fused_bn" -v --timeout 240 --timeout-method thread > gpurun_out/deconv_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/deconv_tests.log | sed 's/tests\/test_gpu_configs.py:://' | head -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/deconv_bench.py > gpurun_out/deconv_v2.txt 2>&1 || exit $?
TIMEONLY=1 bash tools/gpu_train_prof.sh bf16_mfma bf16_norelu bf16_mfma
# config-2 only (B = 4096, graph replays, no sweep / cold / multistream legs): the rocprof
# average of the metric kernel to set beside the bench's event figure
mkdir -p gpurun_out/prof_c2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- python3 bench.py --steps 2000 --warmup 200 --no-cpu-baseline --multistream 1 --cold-launches 0 --no-fwd-bwd --sweep "" > gpurun_out/prof_c2.log 2>&1 || exit $?
grep '^{' gpurun_out/prof_c2.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench events us/launch', d['roofline']['us_per_launch_events'])"
find gpurun_out/prof_c2 -name "*kernel_trace.csv" -delete
