set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py -k "fused_bn or config3 or config4" -q --timeout 240 --timeout-method thread > gpurun_out/bn_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 gpurun_out/bn_tests.log; grep -E "FAILED|ERROR" gpurun_out/bn_tests.log | head
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_train_prof.sh bf16_mfma > gpurun_out/train_ab.log 2>&1 || exit $?
python3 tools/train_kernel_table.py gpurun_out/train_prof/stats_bf16_mfma/run_kernel_stats.csv 24 gpurun_out/train_prof/pmc_bf16_mfma > gpurun_out/train_prof/table_bf16_mfma.txt; head -1 gpurun_out/train_prof/table_bf16_mfma.txt; grep bn_ gpurun_out/train_prof/table_bf16_mfma.txt | cut -c1-120
grep -h '^{' gpurun_out/train_prof/time*_bf16_mfma.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['config']['miopen_find'], round(d['ms_per_step'],3))"
