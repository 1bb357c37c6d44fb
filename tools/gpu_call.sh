#!/bin/bash
# One gpurun call, assembled from named steps (replaces the round-3 one-off call scripts):
#   gpurun -- bash tools/gpu_call.sh tests smoke driver
#   PYTEST_K="bwd or fused" gpurun -- bash tools/gpu_call.sh tests
# Steps:
#   tests        pytest -m gpu (PYTEST_K narrows it with -k)
#   smoke        __graft_entry__.smoke()
#   driver       bench.py in the driver's form (--gpus 1 --steps 20 --warmup 5), summary line
#   c5           bench.py at config 5 (l = 20, B = 8192, bf16 out)
#   sweep        bench.py with the large-batch sweep 16,384 / 65,536 / 262,144
#   prof-c2      tools/gpu_prof.sh c2 (kernel-trace stats + PMC passes, config 2)
#   prof-c5      tools/gpu_prof.sh c5 (same at config 5)
#   prof-driver  rocprofv3 --kernel-trace --stats of the driver-form bench
#   train        bench_train.py config 3, bf16 channels-last, and the fp32 step
#   rehearse     the N-rank rehearsal (two ranks sharing the GPU, gloo)
#   pmc-bwd      PMC passes of the training direction (tools/gpu_pmc_bwd.sh)
#   ab-c5        config-5 bf16 tile-option variants (AB_C5 overrides the list)
#   ab-bwd       backward knob variants (AB_KNOBS, AB_BATCHES override)
# Every GPU step runs under its own time limit; a fault, abort or time-limit kill ends
# the call there (no retries).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  if [ $rc -ne 0 ]; then
    tail -n 30 "$OUT/$name.log"
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] || [ "$name" != pytest_gpu ]; then
      echo "stopping after $name (rc=$rc)"; exit $rc
    fi
  fi
  return 0
}
summary() {  # bench JSON line -> one short line
  grep '^{' "$1" | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; fb=d.get('fwd_bwd') or {}
print('us/launch', round(r['us_per_launch_events'],3), 'raw', round(r['us_per_launch_events_raw'],3),
      'frac', round(r['frac'],4), 'value', round(d['value']/1e6,2), 'M/s')
if fb: print('fwd+bwd graph us', round(fb['us_per_step'],2), 'eager us', round(fb['eager_us_per_step'],1),
             'bwd us', round(fb['action_bwd']['us_per_call'],2))
print('sweep', [(s['batch'], round(s['us'],1), round(s['frac'],3)) for s in (d.get('sweep') or [])])"
}
for s in "$@"; do
  case $s in
    tests)
      if [ -n "${PYTEST_K:-}" ]; then
        step pytest_gpu 900 python -u -m pytest tests -m gpu -v -rf --timeout 240 --timeout-method thread -k "$PYTEST_K"
      else
        step pytest_gpu 900 python -u -m pytest tests -m gpu -v -rf --timeout 240 --timeout-method thread
      fi
      grep -E "passed|failed" "$OUT/pytest_gpu.log" | tail -1
      grep -E "^FAILED|^ERROR" "$OUT/pytest_gpu.log" | head -20 ;;
    smoke)
      step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"; tail -1 "$OUT/smoke.log" ;;
    driver)
      step bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5; summary "$OUT/bench_driver.log" ;;
    c5)
      step bench_c5 600 python bench.py --lmax 20 --batch 8192 --dtype bf16 --no-cpu-baseline --steps 500 --sweep ""
      summary "$OUT/bench_c5.log" ;;
    sweep)
      step bench_sweep 600 python bench.py --no-cpu-baseline --sweep 16384,65536,262144 --no-fwd-bwd
      summary "$OUT/bench_sweep.log" ;;
    prof-c2)
      step prof_c2 900 bash tools/gpu_prof.sh c2 --batch 4096 --lmax 10 --dtype f32 ;;
    prof-c5)
      step prof_c5 900 bash tools/gpu_prof.sh c5 --batch 8192 --lmax 20 --dtype bf16 ;;
    prof-driver)
      step rocprof_driver 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_driver" -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5
      rm -f "$OUT"/prof_driver/*kernel_trace.csv ;;
    train)
      step train_bf16 600 python bench_train.py --global-batch 512 --steps 30 --amp bf16 --channels-last
      grep '^{' "$OUT/train_bf16.log" | cut -c1-240
      step train_f32 600 python bench_train.py --global-batch 512 --steps 20
      grep '^{' "$OUT/train_f32.log" | cut -c1-240 ;;
    rehearse)
      step rehearse 600 bash tools/gpu_rehearse_ranks.sh ;;
    pmc-bwd)
      step pmc_bwd 900 bash tools/gpu_pmc_bwd.sh; cat "$OUT/pmc_bwd.log" ;;
    ab-c5)  # config-5 bf16 tile options (AB_C5 = the variant specs of tools/gpu_variants.sh)
      step ab_c5 900 bash tools/gpu_variants.sh "--lmax 20 --batch 8192 --dtype bf16 --sweep=65536" \
        ${AB_C5:-base= sw5=LV_TILE_SW=5}
      cat "$OUT/ab_c5.log" ;;
    ab-bwd)  # backward knob variants (AB_KNOBS, tools/bwd_reduce_ab.py) at AB_BATCHES
      step ab_bwd 900 env AB_KNOBS="${AB_KNOBS:-LV_BWD_REDUCE=0,LV_BWD_REDUCE=16,LV_BWD_REDUCE=3,LV_BWD_VARIANT=1,LV_BWD_REDUCE=0}" \
        python tools/bwd_reduce_ab.py ${AB_BATCHES:-4096 512 65536}
      cat "$OUT/ab_bwd.log" ;;
    *)
      echo "unknown step $s"; exit 2 ;;
  esac
done
echo "=== done"
