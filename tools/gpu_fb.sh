set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --cold-launches 0 > gpurun_out/bench_fb.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fb -o run --output-format csv -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --cold-launches 0 --multistream 1 > gpurun_out/prof_fb.log 2>&1 || exit $?
rm -f gpurun_out/prof_fb/*kernel_trace.csv
echo done
