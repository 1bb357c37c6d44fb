# Round-3 re-entry: HEAD GPU suite, smoke, driver-form bench, then the forward launch-shape A/B.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v -rf --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -4 gpurun_out/pytest_gpu.log; grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.log 2>&1 || { echo bench failed; tail gpurun_out/bench_driver.log; exit 1; }
grep '^{' gpurun_out/bench_driver.log | tail -1 | cut -c1-1500
bash tools/gpu_fwd_knobs.sh
