set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -k "deconv or relu or conv_dgrad" -q --timeout 240 --timeout-method thread > gpurun_out/deconv_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 gpurun_out/deconv_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/deconv_bench.py > gpurun_out/deconv_v2c.txt 2>&1 || exit $?
grep '^{' gpurun_out/deconv_v2c.txt | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print({k:(round(v,1) if isinstance(v,float) else v) for k,v in d.items() if k.endswith('_us') or 'bitwise' in k or k=='H_in'})"
