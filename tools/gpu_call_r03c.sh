set -u
mkdir -p gpurun_out
timeout -k 10 60 python tools/event_probe.py > gpurun_out/event_probe2.txt 2>&1; echo "probe rc=$?"; grep -v amdgpu.ids gpurun_out/event_probe2.txt
bash tools/gpu_train_prof.sh bf16 f32
