"""A/B of backward tile-kernel builds (register budget) x degree-segment count.

Each (library, nseg) runs in its own process: LIEVAE_HIP_LIB picks the build,
LV_BWD_NSEG forces the segment count (the libraries must be A/B builds, -DLV_AB_KNOBS:
the product library reads no environment).  Prints us/call of lv_group_action_bwd at
batch 4096, l = 10, C = 10 and a hash of (gang, gF) so that builds can be checked
bit for bit against each other.
  python tools/bwd_variant_sweep.py lib1.so lib2.so ...
"""
import json
import os
import subprocess
import sys

CHILD = r"""
import os, sys, json, hashlib, ctypes, torch
sys.path[:0] = ['lie-vae_amd', '.']
import bench
from lie_vae import _lib
dev = torch.device('cuda:0')
torch.manual_seed(0)
L, C = 10, 10
B = int(os.environ.get('SWEEP_B', '4096'))
v = torch.randn(B, 3, device=dev); F = torch.randn(121, C, device=dev)
g = torch.randn(B, 121, C, device=dev)
r = bench.bench_action_bwd_kernel(v, F, g, L, dev, reps=400)
lib = _lib.load()
import lie_vae._ops as ops
ang = torch.empty(B, 3, device=dev)
out = torch.empty(B, 121, C, device=dev)
P = lambda t: ctypes.c_void_p(t.data_ptr())
lib.lv_fused_exp_action_fwd(None, P(v), P(F), 0, P(out), _lib.LV_DTYPE_F32, P(ang), B, L, C, 0, None)
gang = torch.empty(B, 3, device=dev); gF = torch.empty(121, C, device=dev)
wsb = lib.lv_group_action_bwd_workspace(B, L, C, 1)
ws = torch.empty(max(wsb, 1), device=dev, dtype=torch.uint8)
rc = lib.lv_group_action_bwd(P(ang), P(F), 0, P(g), P(gang), P(gF), B, L, C, 0, P(ws), wsb, None)
assert rc == 0, _lib.last_error()
torch.cuda.synchronize()
h = hashlib.sha1(gang.cpu().numpy().tobytes() + gF.cpu().numpy().tobytes()).hexdigest()[:16]
print(json.dumps({"us": r["us_per_call"], "hash": h}))
"""


def main():
    libs = sys.argv[1:]
    for lib in libs:
        for ns in [int(x) for x in os.environ.get('SWEEP_NSEG', '2,3,4,6,8').split(',')]:
            env = dict(os.environ, LV_BWD_NSEG=str(ns), LIEVAE_HIP_LIB=os.path.abspath(lib))
            try:
                r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True,
                                   text=True, timeout=120)
            except subprocess.TimeoutExpired:
                print(os.path.basename(lib), ns, "TIMEOUT", flush=True)
                return 1
            if r.returncode != 0:
                print(os.path.basename(lib), ns, "rc", r.returncode, r.stderr[-400:], flush=True)
                if r.returncode < 0 or r.returncode in (134, 139):
                    return 1
                continue
            print(os.path.basename(lib), ns, r.stdout.strip().splitlines()[-1], flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
