set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py -k "config3 or config4 or dp_trainer" -q --timeout 240 --timeout-method thread > gpurun_out/adam_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 gpurun_out/adam_tests.log; grep -E "FAILED|ERROR" gpurun_out/adam_tests.log | head
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_train_prof.sh bf16_foreach bf16_mfma > gpurun_out/train_ab.log 2>&1 || exit $?
for v in mfma foreach; do python3 tools/train_kernel_table.py gpurun_out/train_prof/stats_bf16_$v/run_kernel_stats.csv 24 gpurun_out/train_prof/pmc_bf16_$v > gpurun_out/train_prof/table_bf16_$v.txt; head -1 gpurun_out/train_prof/table_bf16_$v.txt; done
grep -h '^{' gpurun_out/train_prof/time*_bf16_{mfma,foreach}.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['config'].get('adam'), d['config']['miopen_find'], round(d['ms_per_step'],3))"
