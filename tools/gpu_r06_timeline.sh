set -u
mkdir -p gpurun_out
LIEVAE_HIP_LIB=$PWD/lie-vae_amd/lie_vae/liblievae_hip_ab.so LV_STAMPS=1 timeout -k 10 120 python tools/timeline.py 4096 10 f32 fwd > gpurun_out/tl_fwd.txt 2>&1; echo tl rc=$?; grep -v amdgpu.ids gpurun_out/tl_fwd.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread -k "other_grid_sizes" > gpurun_out/t_grid.log 2>&1; echo "pytest rc=$?"; grep -E "passed|failed|^E  " gpurun_out/t_grid.log | tail -5
