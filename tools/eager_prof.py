"""Host cost of the eager training direction at config 2 (bench.py fwd_bwd's step):
wall time per step with the GPU running behind (host-bound when above the graph time),
then a cProfile of the same loop (top entries by own time).
  python tools/eager_prof.py"""
import cProfile
import os
import pstats
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "lie-vae_amd"), REPO]
import lie_vae._ops as ops  # noqa: E402

dev = torch.device("cuda:0")
B, L, C = 4096, 10, 10
v = torch.randn(B, 3, device=dev).requires_grad_(True)
F = torch.randn((L + 1) ** 2, C, device=dev).requires_grad_(True)
gout = torch.randn(B, (L + 1) ** 2, C, device=dev)


def step():
    v.grad = None
    F.grad = None
    ops.fused_exp_action(None, v, F, L).backward(gout)


def fwd_only():
    with torch.no_grad():
        ops.fused_exp_action(None, v, F, L)


for fn, tag in ((step, "fwd+bwd"), (fwd_only, "fwd")):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    n = 500
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{tag}: host {1e6 * (t1 - t0) / n:.1f} us/step, wall {1e6 * (t2 - t0) / n:.1f} us/step", flush=True)
pr = cProfile.Profile()
pr.enable()
for _ in range(300):
    step()
pr.disable()
torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
