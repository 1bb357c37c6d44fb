# Round-6 evidence at HEAD: driver-form bench line, its rocprofv3 kernel stats, the
# config-2 / config-5 kernel stats + PMC (tools/gpu_prof.sh), PMC and kernel traces of the
# backward alone at 4,096 and 65,536 (tools/bwd_only.py), for profiles/r06_*.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/ev_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 8 "gpurun_out/ev_$name.log"; exit $rc; fi
}
if [ "${PART:-1}" = 1 ]; then
step bench 300 python bench.py --gpus 1 --steps 20 --warmup 5
step rocprof_driver 400 rocprofv3 --kernel-trace --stats -d gpurun_out/ev_prof_driver -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5
rm -f gpurun_out/ev_prof_driver/*kernel_trace.csv
for B in 4096 65536; do
  step bwd_trace_$B 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ev_bwd_$B -o run --output-format csv -- python3 tools/bwd_only.py $B 20
  rm -f gpurun_out/ev_bwd_$B/*kernel_trace.csv
  step pmc_bwd_$B 400 bash tools/gpu_pmc_bwd_only.sh $B action_bwd_persist
done
echo "=== part 1 done"; exit 0
fi
step bench2 300 python bench.py --gpus 1 --steps 20 --warmup 5
step prof_c2 600 bash tools/gpu_prof.sh c2 --batch 4096 --lmax 10 --dtype f32
step prof_c5 600 bash tools/gpu_prof.sh c5 --batch 8192 --lmax 20 --dtype bf16
echo "=== done"
