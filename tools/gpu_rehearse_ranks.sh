#!/bin/bash
# Rehearsal of the N-rank bench paths on a one-GPU box (LV_SHARE_GPU0=1: every rank on
# cuda:0, gloo instead of RCCL).  Checks the launcher hand-off, the driver-style
# torch.distributed.run start, barriers and max-over-ranks timing; numbers are not
# scaling results (two ranks share one GPU).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export LV_SHARE_GPU0=1
timeout -k 10 300 python bench.py --gpus 2 --steps 500 --warmup 50 --no-cpu-baseline --cold-launches 0 --no-fwd-bwd > gpurun_out/rehearse_bench_self.log 2>&1 || { echo "self-launch rc=$?"; tail -20 gpurun_out/rehearse_bench_self.log; exit 1; }
tail -1 gpurun_out/rehearse_bench_self.log | cut -c1-400
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 500 --warmup 50 --no-cpu-baseline --cold-launches 0 --no-fwd-bwd > gpurun_out/rehearse_bench_torchrun.log 2>&1 || { echo "torchrun rc=$?"; tail -20 gpurun_out/rehearse_bench_torchrun.log; exit 1; }
grep '^{' gpurun_out/rehearse_bench_torchrun.log | cut -c1-400
timeout -k 10 400 python bench_train.py --gpus 2 --global-batch 1024 --steps 5 --warmup 2 > gpurun_out/rehearse_train.log 2>&1 || { echo "train rc=$?"; tail -20 gpurun_out/rehearse_train.log; exit 1; }
grep '^{' gpurun_out/rehearse_train.log | cut -c1-400
echo done
