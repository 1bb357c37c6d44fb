"""A/B of the shared-spectrum dF reduction of lv_group_action_bwd (A/B build knob
LV_BWD_REDUCE: 1 = action_bwd_reduce_kernel (round 2), 4 / 8 / 16 = action_bwd_reduce2_kernel<COLS>,
16 the default since round 3; the first table, profiles/r03_bwd_reduce_ab.txt, was taken when 0 = the
round-2 kernel was the default).
Per variant (own process): us per lv_group_action_bwd call at batch B (graph-captured,
bench.bench_action_bwd_kernel), gF against the default kernel (relative max error) and
a repeat call bit for bit.
  python tools/bwd_reduce_ab.py [B ...]
"""
import json
import os
import subprocess
import sys

CHILD = r"""
import os, sys, json, ctypes, torch, numpy as np
sys.path[:0] = ['lie-vae_amd', '.']
import bench
from lie_vae import _lib
dev = torch.device('cuda:0')
torch.manual_seed(0)
L, C = 10, 10
B = int(sys.argv[1])
v = torch.randn(B, 3, device=dev); F = torch.randn(121, C, device=dev)
g = torch.randn(B, 121, C, device=dev)
r = bench.bench_action_bwd_kernel(v, F, g, L, dev, reps=400)
lib = _lib.load()
ang = torch.empty(B, 3, device=dev)
out = torch.empty(B, 121, C, device=dev)
P = lambda t: ctypes.c_void_p(t.data_ptr())
lib.lv_fused_exp_action_fwd(None, P(v), P(F), 0, P(out), _lib.LV_DTYPE_F32, P(ang), B, L, C, 0, None)
wsb = lib.lv_group_action_bwd_workspace(B, L, C, 1)
ws = torch.empty(max(wsb, 1), device=dev, dtype=torch.uint8)
res = []
for _ in range(2):
    gang = torch.empty(B, 3, device=dev); gF = torch.empty(121, C, device=dev)
    rc = lib.lv_group_action_bwd(P(ang), P(F), 0, P(g), P(gang), P(gF), B, L, C, 0, P(ws), wsb, None)
    assert rc == 0, _lib.last_error()
    torch.cuda.synchronize()
    res.append(gF.cpu().numpy())
np.save(sys.argv[2], res[0])
print(json.dumps({"us": r["us_per_call"], "repeat_bitwise": bool(np.array_equal(res[0], res[1]))}))
"""


def main():
    batches = [int(x) for x in sys.argv[1:]] or [4096, 512, 65536]
    os.makedirs("gpurun_out", exist_ok=True)
    for B in batches:
        ref = None
        knobs = os.environ.get("AB_KNOBS", "LV_BWD_REDUCE=1,LV_BWD_REDUCE=16,LV_BWD_REDUCE=8,LV_BWD_REDUCE=4,LV_BWD_REDUCE=1")
        for kv in knobs.split(","):
            # one variant: NAME=val, or several joined by '+' (NAME=val+NAME2=val2)
            pairs = dict(x.split("=") for x in kv.split("+"))
            name, knob = "+".join(pairs), "+".join(pairs.values())
            path = f"gpurun_out/gF_{B}_{kv.replace('+', '_')}.npy"
            env = dict(os.environ, **pairs,
                       LIEVAE_HIP_LIB=os.path.abspath("lie-vae_amd/lie_vae/liblievae_hip_ab.so"))
            r = subprocess.run([sys.executable, "-c", CHILD, str(B), path], env=env,
                               capture_output=True, text=True, timeout=120)
            if r.returncode != 0:
                print(B, name, knob, "rc", r.returncode, r.stderr[-600:], flush=True)
                return 1
            d = json.loads(r.stdout.strip().splitlines()[-1])
            import numpy as np
            gF = np.load(path)
            if ref is None:
                ref = gF
            err = float(np.abs(gF - ref).max() / np.abs(ref).max())
            print(f"B={B:6d} {name}={knob:>2}: {d['us']:7.2f} us/call  repeat bitwise {d['repeat_bitwise']}"
                  f"  max |gF - default| / max|gF| {err:.2e}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
