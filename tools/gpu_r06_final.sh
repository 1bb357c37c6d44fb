# Round-6 check at HEAD after the forward degree-set change (kDegFixedFwd 80): the GPU
# test suite, smoke(), the driver-form bench line, and the config-2 degree-set A/B of the
# planner's sets against the previous ones (LV_TILE_MASKS, A/B library).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/fin_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 12 "gpurun_out/fin_$name.log"; exit $rc; fi
}
step pytest 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 300 python bench.py --gpus 1 --steps 20 --warmup 5
step ab_masks 400 bash tools/gpu_variants.sh "--batch 4096 --lmax 10 --dtype f32 --sweep=65536" plan= old=LV_TILE_MASKS=400:200:102:84:48:31 plan2= old2=LV_TILE_MASKS=400:200:102:84:48:31
tail -n 1 gpurun_out/fin_bench.log
cat gpurun_out/fin_ab_masks.log
echo "=== done"
