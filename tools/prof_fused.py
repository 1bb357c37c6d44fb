"""Minimal driver for profiling the fused action kernel: R launches at batch B."""
import ctypes
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lie-vae_amd"))
from lie_vae import _lib  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
R = int(sys.argv[2]) if len(sys.argv) > 2 else 200
L = int(sys.argv[3]) if len(sys.argv) > 3 else 10
C = int(sys.argv[4]) if len(sys.argv) > 4 else 10
fused = int(os.environ.get("LV_FUSED", "1"))
bf16 = int(os.environ.get("LV_BF16", "0"))  # output dtype (config 5: bf16)
lib = _lib.load()
dev = torch.device("cuda:0")
M = (L + 1) ** 2
v = torch.randn(B, 3, device=dev)
ang = torch.rand(B, 3, device=dev)
F = torch.randn(M, C, device=dev)
out = torch.empty(B, M, C, device=dev, dtype=torch.bfloat16 if bf16 else torch.float32)
dt = _lib.LV_DTYPE_BF16 if bf16 else _lib.LV_DTYPE_F32
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
for _ in range(R):
    if fused:
        rc = lib.lv_fused_exp_action_fwd(None, P(v), P(F), 0, P(out), dt, None, B, L, C, 0, s)
    else:
        rc = lib.lv_group_action_fwd(P(ang), P(F), 0, P(out), dt, B, L, C, 0, s)
    assert rc == 0, _lib.last_error()
torch.cuda.synchronize()
print("ok", B, R, L, C)
