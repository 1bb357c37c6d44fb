set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -k "mfma_deconv_backward" -q --timeout 200 --timeout-method thread > gpurun_out/deconv_test.log 2>&1; rc=$?; echo "deconv tests rc=$rc"; grep -E "passed|failed|Error|assert|off," gpurun_out/deconv_test.log | head -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/deconv_bwd_bench.py > gpurun_out/deconv_bwd_bench.txt 2>&1; echo "deconv bwd bench rc=$?"; grep -v amdgpu gpurun_out/deconv_bwd_bench.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dbwd -o run --output-format csv -- python3 tools/deconv_bwd_bench.py > gpurun_out/prof_dbwd.log 2>&1; echo "prof rc=$?"
python3 - <<'PY'
import csv,glob
f=glob.glob("gpurun_out/prof_dbwd/**/run_kernel_stats.csv",recursive=True)[0]
for r in sorted(csv.DictReader(open(f)), key=lambda r:-float(r["TotalDurationNs"]))[:14]:
    print(f'{float(r["AverageNs"])/1e3:9.2f} us x{r["Calls"]:>5}  {r["Name"][:100]}')
PY
