set -u
mkdir -p gpurun_out
for n in 4096 16384 65536 262144; do
  timeout -k 10 120 ./tools/kbench_fwd $n $((4000000 / n + 50)) > gpurun_out/fwd_occ_B$n.txt 2>&1 || { echo "fwd $n failed"; exit 1; }
  grep -E "nomu|lib tile" gpurun_out/fwd_occ_B$n.txt
done
timeout -k 10 200 ./tools/kbench_c5 8192 200 mreg > gpurun_out/c5_nomu.txt 2>&1; echo "c5 rc=$?"; cat gpurun_out/c5_nomu.txt
