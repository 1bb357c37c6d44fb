set -u
mkdir -p gpurun_out
timeout -k 10 300 ./tools/kbench_c5 8192 200 ab > gpurun_out/c5_tile2.txt 2>&1; echo "c5 rc=$?"; cat gpurun_out/c5_tile2.txt
