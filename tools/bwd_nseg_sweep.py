import os, sys, json, subprocess
res = {}
for ns in [1, 2, 3, 4]:
    env = dict(os.environ, LV_BWD_NSEG=str(ns),
               LIEVAE_HIP_LIB=os.path.abspath("lie-vae_amd/lie_vae/liblievae_hip_ab.so"))  # knobs: A/B build only
    r = subprocess.run([sys.executable, "-c", """
import sys, json, torch
sys.path[:0] = ['lie-vae_amd', '.']
import bench
dev = torch.device('cuda:0')
torch.manual_seed(0)
L, C, B = 10, 10, 4096
v = torch.randn(B, 3, device=dev); F = torch.randn(121, C, device=dev); g = torch.randn(B, 121, C, device=dev)
print(json.dumps(bench.bench_action_bwd_kernel(v, F, g, L, dev, reps=400)))
"""], env=env, capture_output=True, text=True, timeout=120)
    res[ns] = r.stdout.strip().splitlines()[-1] if r.returncode == 0 else r.stderr[-500:]
    print(ns, res[ns], flush=True)
