set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -1 gpurun_out/pytest_gpu.log; grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head -10
[ $rc -le 1 ] || exit $rc
bash tools/gpu_fwd_knobs.sh
AB_KNOBS="LV_BWD_PRIO=0,LV_BWD_PRIO=2,LV_BWD_PRIO=0,LV_BWD_PRIO=2" timeout -k 10 400 python tools/bwd_reduce_ab.py 4096 16384 65536 > gpurun_out/bwd_prio_ab.txt 2>&1; cat gpurun_out/bwd_prio_ab.txt
