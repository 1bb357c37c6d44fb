# fp32 MFMA deconv kernel variants (A/B library, LV_DECONV_F32_VARIANT: 1 = 128-row tiles, 2
# stages; 2 = 128 rows, 3 stages; 3 = 256 rows, 2 stages; 4 = 256 rows, 3 stages): the
# per-layer timing of tools/deconv_f32_bench.py and the parity tests for each.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
export LIEVAE_HIP_LIB=$PWD/lie-vae_amd/lie_vae/liblievae_hip_ab.so
for v in 1 2 3 4 1; do
  echo "== variant $v"
  LV_DECONV_F32_VARIANT=$v timeout -k 10 200 python -u -m pytest tests/test_gpu_configs.py -x -q --timeout 100 --timeout-method thread -k "f32_matches_float64" > gpurun_out/dcf32_t$v.log 2>&1 || { echo "tests failed v=$v"; tail -20 gpurun_out/dcf32_t$v.log; exit 1; }
  tail -n 1 gpurun_out/dcf32_t$v.log
  LV_DECONV_F32_VARIANT=$v timeout -k 10 200 python -u tools/deconv_f32_bench.py > gpurun_out/dcf32_b$v.log 2>&1 || { echo "bench failed v=$v"; tail -5 gpurun_out/dcf32_b$v.log; exit 1; }
  python3 -c "
import json,sys
for l in open('gpurun_out/dcf32_b$v.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['layer'], 'miopen %.0f us' % d['miopen_us'], 'kernel %.0f us %.1f TF' % (d['mfma_f32_kernel_us'], d['gflop']/d['mfma_f32_kernel_us']*1e3), 'path %.0f' % d['mfma_f32_path_us'])
"
done
