# Persistent backward: the padded gradient tile (conflict-free chain reads) moved by buffer
# loads to LDS (variant 7713 = product 6689 + kBwdVarPersistPad) against the product; its
# parity tests on the A/B library; its PMC at 65,536 (LDS bank conflicts per LDS instruction).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_KNOBS="LV_BWD_VARIANT=6689,LV_BWD_VARIANT=7713,LV_BWD_VARIANT=6689,LV_BWD_VARIANT=7713" \
  timeout -k 10 600 python -u tools/bwd_reduce_ab.py 65536 262144 4096 16384 > gpurun_out/ab_padbuf.log 2>&1 || { echo ab failed; tail -20 gpurun_out/ab_padbuf.log; exit 1; }
cat gpurun_out/ab_padbuf.log
LIEVAE_HIP_LIB=$PWD/lie-vae_amd/lie_vae/liblievae_hip_ab.so LV_BWD_VARIANT=7713 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread -k "persistent or shared_spectrum or reproducible or fused_exp_action_bwd" > gpurun_out/t_padbuf.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/t_padbuf.log | tail -3
[ $rc -eq 0 ] || { grep FAIL gpurun_out/t_padbuf.log | head; exit $rc; }
LIEVAE_HIP_LIB=$PWD/lie-vae_amd/lie_vae/liblievae_hip_ab.so LV_BWD_VARIANT=7713 timeout -k 10 600 bash tools/gpu_pmc_bwd_only.sh 65536 action_bwd_persist > gpurun_out/pmc_padbuf.log 2>&1 || { echo pmc failed; tail -10 gpurun_out/pmc_padbuf.log; exit 1; }
rm -rf gpurun_out/pmc_bwd_only_65536_v7713; mv gpurun_out/pmc_bwd_only_65536 gpurun_out/pmc_bwd_only_65536_v7713
cat gpurun_out/pmc_bwd_only_65536_v7713/summary.txt
