# HEAD: full GPU suite, smoke, driver bench, N-rank rehearsal (bf16 DP training with the new layers)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -v -rf --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -1 gpurun_out/pytest_gpu.log; grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
bash tools/gpu_rehearse_ranks.sh
LV_SHARE_GPU0=1 timeout -k 10 400 python bench_train.py --gpus 2 --global-batch 1024 --steps 5 --warmup 2 --amp bf16 --channels-last > gpurun_out/rehearse_train_bf16.log 2>&1 || { echo "bf16 train rc=$?"; tail -20 gpurun_out/rehearse_train_bf16.log; exit 1; }
grep '^{' gpurun_out/rehearse_train_bf16.log | cut -c1-300
