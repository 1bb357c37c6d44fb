#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprof (+ optional PMC / calibration).
# Every GPU step has its own time limit; a fault/abort/timeout ends the script there.
#   bash tools/gpu_round.sh [all|test|bench|prof]
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
OUT=gpurun_out
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 25 "$OUT/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "fatal rc=$rc in $name; stopping"; exit $rc
  fi
  return 0
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = test ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -v -rf --timeout 240 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5
  step bench 600 python bench.py --sweep 16384,65536,262144
  step bench_c5 600 python bench.py --lmax 20 --batch 8192 --dtype bf16 --no-cpu-baseline --steps 500
  cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
  step rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 300 --warmup 50 --no-cpu-baseline --multistream 1 --cold-launches 0 --no-fwd-bwd
  rm -f "$OUT"/prof/*kernel_trace.csv
  step rocprof_driver 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_driver" -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5
  rm -f "$OUT"/prof_driver/*kernel_trace.csv
fi
if [ "$MODE" = all ] || [ "$MODE" = train ]; then
  step train_c3 600 python bench_train.py --global-batch 512 --steps 20
  cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
  step prof_train 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_train" -o run --output-format csv -- python3 bench_train.py --steps 10 --warmup 3
  rm -f "$OUT"/prof_train/*kernel_trace.csv
fi
if [ "$MODE" = prof ] || [ "$MODE" = traffic ]; then
  cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
  step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_tr/fetch" -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --launch eager --multistream 1
  step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_tr/write" -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --launch eager --multistream 1
  step traffic 60 python3 tools/pmc_traffic.py "$OUT/pmc_tr" "$OUT/traffic_B4096_L10_C10_f32.json"
fi
if [ "$MODE" = prof ]; then
  cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
  for g in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT"; do
    tag=$(echo $g | cut -d' ' -f1)
    step pmc_$tag 300 rocprofv3 --pmc $g --output-format csv -d "$OUT/pmc/$tag" -o run -- python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline --launch eager
  done
  step pmc_summary 60 python3 tools/pmc_summary.py "$OUT/pmc" action_fwd
  step storebench 120 ./tools/kbench_store 4096
fi
echo "=== done"
