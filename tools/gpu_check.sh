# Check at HEAD: the GPU test suite, smoke(), the default bench line (gpurun_out/fin2_*.log).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/fin2_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 15 "gpurun_out/fin2_$name.log"; exit $rc; fi
}
step pytest 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
tail -n 1 gpurun_out/fin2_pytest.log
step smoke 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 300 python bench.py
tail -n 1 gpurun_out/fin2_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); t=d['train_step']; print('value', d['value'], 'us', d['roofline']['us_per_launch_events'], 'frac', d['roofline']['frac'], 'c5', d['config5']['us_per_launch'], 'train', t['bf16']['ms_per_step_rounds'], t['f32']['ms_per_step_rounds'])"
