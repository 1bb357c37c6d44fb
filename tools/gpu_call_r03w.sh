set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py -k "deconv or relu" -v --timeout 240 --timeout-method thread > gpurun_out/deconv_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/deconv_tests.log | sed 's/tests\/test_gpu_configs.py:://' | grep -v "PASSED" | head; grep -c PASSED gpurun_out/deconv_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_train_prof.sh bf16_mfma bf16_norelu > gpurun_out/train_ab.log 2>&1 || exit $?
for v in mfma norelu; do python3 tools/train_kernel_table.py gpurun_out/train_prof/stats_bf16_$v/run_kernel_stats.csv 24 gpurun_out/train_prof/pmc_bf16_$v | head -1; done
grep -h '^{' gpurun_out/train_prof/time*_bf16_*.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['config']['fused_relu'], d['config']['miopen_find'], round(d['ms_per_step'],3))"
