"""Where the eager forward + backward step's host time goes (config 2, B = 4,096):
wall time per step of successively larger pieces, each a loop of 300 after warm-up,
synchronised once at the end (so a GPU-bound piece shows its kernel time and a host-
bound piece its host time).  A/B tool; prints one line per piece."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lie-vae_amd"))
import lie_vae._ops as ops  # noqa: E402
from lie_vae import _lib  # noqa: E402

dev = torch.device("cuda:0")
B, L, C = 4096, 10, 10
M = (L + 1) ** 2
v = torch.randn(B, 3, device=dev)
F = torch.randn(M, C, device=dev)
vg = v.clone().requires_grad_(True)
Fg = F.clone().requires_grad_(True)
gout = torch.randn(B, M, C, device=dev)
out_buf = torch.empty(B, M, C, device=dev)
ang = torch.empty(B, 3, device=dev)


def timeit(name, fn, n=300):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    print(f"{name:>48}: {(time.perf_counter() - t0) / n * 1e6:7.1f} us/step", flush=True)


st = _lib.stream_of(dev)
timeit("C-ABI forward launch only (ctypes)", lambda: _lib.call(
    "lv_fused_exp_action_fwd", None, v.data_ptr(), F.data_ptr(), 0, out_buf.data_ptr(), 0, ang.data_ptr(),
    B, L, C, 0, st))
timeit("torch.empty x2", lambda: (torch.empty(B, M, C, device=dev), torch.empty(B, 3, device=dev)))
with torch.no_grad():
    timeit("op forward, no grad (torch.ops)", lambda: torch.ops.lievae.fused_exp_action(None, v, F, L, False, False))
    timeit("ops.fused_exp_action wrapper, no grad", lambda: ops.fused_exp_action(None, v, F, L))
timeit("op forward with autograd record", lambda: torch.ops.lievae.fused_exp_action(None, vg, Fg, L, False, False))


def step_op():
    vg.grad = None
    Fg.grad = None
    torch.ops.lievae.fused_exp_action(None, vg, Fg, L, False, False).backward(gout)


def step_wrap():
    vg.grad = None
    Fg.grad = None
    ops.fused_exp_action(None, vg, Fg, L).backward(gout)


def step_grad():
    o = torch.ops.lievae.fused_exp_action(None, vg, Fg, L, False, False)
    torch.autograd.grad(o, (vg, Fg), gout)


timeit("fwd + bwd (torch.ops, .backward)", step_op)
timeit("fwd + bwd (wrapper, .backward) = bench eager", step_wrap)
timeit("fwd + bwd (torch.ops, autograd.grad)", step_grad)
x = torch.randn(16, device=dev, requires_grad=True)
timeit("tiny torch op fwd + bwd (x*2).sum().backward()", lambda: (x * 2).sum().backward())
