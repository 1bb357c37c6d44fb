# Persistent backward: the dF slab as whole 16-byte write-through (sc1) stores (variant 23073 =
# product 6689 + kBwdVarPersistSlabWT) against the product; parity tests on the A/B library.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_KNOBS="LV_BWD_VARIANT=6689,LV_BWD_VARIANT=23073,LV_BWD_VARIANT=6689,LV_BWD_VARIANT=23073" \
  timeout -k 10 600 python -u tools/bwd_reduce_ab.py 4096 65536 16384 2048 > gpurun_out/ab_slabwt.log 2>&1 || { echo ab failed; tail -20 gpurun_out/ab_slabwt.log; exit 1; }
cat gpurun_out/ab_slabwt.log
LIEVAE_HIP_LIB=$PWD/lie-vae_amd/lie_vae/liblievae_hip_ab.so LV_BWD_VARIANT=23073 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread -k "persistent or shared_spectrum or reproducible or fused_exp_action_bwd" > gpurun_out/t_slabwt.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/t_slabwt.log | tail -3; exit $rc
