# PMC (MFMA busy, LDS) and kernel stats of the fp32 MFMA deconv kernel on the 16 -> 32 layer (B = 512)
set -u
mkdir -p gpurun_out/pmc_dcf32
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/pmc_dcf32/p1 -o run -- python3 tools/deconv_f32_bench.py 16 > gpurun_out/pmc_dcf32/p1.log 2>&1 || { echo p1 failed; tail -5 gpurun_out/pmc_dcf32/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc_dcf32/st -o run -- python3 tools/deconv_f32_bench.py 16 > gpurun_out/pmc_dcf32/st.log 2>&1 || { echo st failed; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmc_dcf32/p1 deconv_mfma_f32 > gpurun_out/pmc_dcf32/summary.txt
grep deconv_mfma_f32 gpurun_out/pmc_dcf32/st/run_kernel_stats.csv | cut -c1-200 >> gpurun_out/pmc_dcf32/summary.txt
find gpurun_out/pmc_dcf32 -name "*counter_collection.csv" -size +2M -delete
rm -f gpurun_out/pmc_dcf32/st/*kernel_trace.csv
cat gpurun_out/pmc_dcf32/summary.txt
