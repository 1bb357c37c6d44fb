# HEAD after removing the persistent / split kernels: GPU suite, reduce A/B, round-3 evidence
# (driver-form bench, rocprof kernel stats, PMC HBM traffic for config 2 and config 5).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { echo "fatal rc=$1 in $2"; exit $1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -v -rf --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -2 gpurun_out/pytest_gpu.log; grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head -20
[ $rc -le 1 ] || fatal $rc pytest
timeout -k 10 400 python tools/bwd_reduce_ab.py 4096 512 65536 > gpurun_out/bwd_reduce_ab.txt 2>&1; rc=$?; cat gpurun_out/bwd_reduce_ab.txt; [ $rc -eq 0 ] || fatal $rc reduce_ab
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.log 2>&1 || fatal $? bench_driver
grep '^{' gpurun_out/bench_driver.log | tail -1 | cut -c1-400
timeout -k 10 300 python bench.py --lmax 20 --batch 8192 --dtype bf16 --no-cpu-baseline --steps 500 --sweep 65536 > gpurun_out/bench_c5.log 2>&1 || fatal $? bench_c5
rm -rf gpurun_out/prof gpurun_out/pmc_tr gpurun_out/pmc_tr5
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/rocprof_driver.log 2>&1 || fatal $? rocprof
find gpurun_out/prof -name "*kernel_trace.csv" -delete
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_tr/fetch -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --launch eager --multistream 1 --no-fwd-bwd --cold-launches 0 --sweep "" > gpurun_out/pmc1.log 2>&1 || fatal $? pmc_fetch
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_tr/write -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --launch eager --multistream 1 --no-fwd-bwd --cold-launches 0 --sweep "" > gpurun_out/pmc2.log 2>&1 || fatal $? pmc_write
python3 tools/pmc_traffic.py gpurun_out/pmc_tr gpurun_out/traffic_B4096_L10_C10_f32.json
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_tr5/fetch -o run -- python3 bench.py --lmax 20 --batch 8192 --dtype bf16 --steps 100 --warmup 20 --no-cpu-baseline --launch eager --multistream 1 --no-fwd-bwd --cold-launches 0 --sweep "" > gpurun_out/pmc3.log 2>&1 || fatal $? pmc5_fetch
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_tr5/write -o run -- python3 bench.py --lmax 20 --batch 8192 --dtype bf16 --steps 100 --warmup 20 --no-cpu-baseline --launch eager --multistream 1 --no-fwd-bwd --cold-launches 0 --sweep "" > gpurun_out/pmc4.log 2>&1 || fatal $? pmc5_write
python3 tools/pmc_traffic.py gpurun_out/pmc_tr5 gpurun_out/traffic_B8192_L20_C10_bf16.json
find gpurun_out/pmc_tr gpurun_out/pmc_tr5 -name "*counter_collection.csv" -size +20M -delete
echo done
