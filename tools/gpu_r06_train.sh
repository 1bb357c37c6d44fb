set -u
mkdir -p gpurun_out/trainprof
export TMPDIR=/tmp
timeout -k 10 300 python bench_train.py --global-batch 512 --steps 30 --amp bf16 --channels-last > gpurun_out/train_bf16_a.log 2>&1; echo a rc=$?; grep '^{' gpurun_out/train_bf16_a.log | cut -c1-300
timeout -k 10 300 python bench_train.py --global-batch 512 --steps 30 --amp bf16 --channels-last > gpurun_out/train_bf16_b.log 2>&1; echo b rc=$?; grep '^{' gpurun_out/train_bf16_b.log | cut -c1-300
cd /tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/trainprof -o run --output-format csv -- python3 bench_train.py --global-batch 512 --steps 20 --warmup 5 --amp bf16 --channels-last > gpurun_out/train_prof.log 2>&1; echo prof rc=$?
find gpurun_out/trainprof -name "*kernel_trace.csv" -delete
