#!/bin/bash
# Round-5 evidence at HEAD: GPU tests + smoke, the driver-form bench line and its rocprofv3
# kernel stats, config-2 and config-5 rocprof + PMC (tools/gpu_prof.sh), the backward alone
# at 4,096 / 65,536 (kernel trace).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1; shift; echo "=== $name $(date +%T)"; "$@"; local rc=$?; echo "=== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step tests timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench sh -c "timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05_bench_driver.json 2> gpurun_out/r05_bench_driver.err"
step bench_prof timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_prof_driver -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5
rm -f gpurun_out/r05_prof_driver/*kernel_trace.csv
step prof_c2 bash tools/gpu_prof.sh c2 --batch 4096 --lmax 10 --dtype f32
step prof_c5 bash tools/gpu_prof.sh c5 --batch 8192 --lmax 20 --dtype bf16
for B in 4096 65536; do
  step bwd_$B timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_bwd_only_$B -o run --output-format csv -- python3 tools/bwd_only.py $B
  rm -f gpurun_out/r05_bwd_only_$B/*kernel_trace.csv
done
# the N > 1 code path (config 4's DP train record, RCCL replaced by gloo because two ranks
# share the box's one GPU): plumbing only, not scaling numbers
step rehearse2 sh -c "LV_SHARE_GPU0=1 timeout -k 10 400 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline --sweep= --cold-launches 0 > gpurun_out/r05_rehearse_2ranks.json 2> gpurun_out/r05_rehearse_2ranks.err"
echo "=== all done"
