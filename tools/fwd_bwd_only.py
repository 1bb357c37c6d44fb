#!/usr/bin/env python3
"""The bench's fwd_bwd record alone: the fused forward + autograd backward at config 2
(B = 4,096, l = 10, C = 10), captured once in a hipGraph and replayed, for a kernel trace
of exactly one training-direction step:

  rocprofv3 --kernel-trace --stats -d gpurun_out/p -o run -- python3 tools/fwd_bwd_only.py
"""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "lie-vae_amd"), REPO]


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    L, C = 10, 10
    import lie_vae._ops as ops
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(3)
    vg = torch.randn(B, 3, generator=g).to(dev).requires_grad_(True)
    Fg = torch.randn((L + 1) ** 2, C, generator=g).to(dev).requires_grad_(True)
    gout = torch.randn(B, (L + 1) ** 2, C, generator=g).to(dev)
    side = torch.cuda.Stream(dev)
    with torch.cuda.stream(side):
        for _ in range(3):
            vg.grad = None
            Fg.grad = None
            ops.fused_exp_action(None, vg, Fg, L).backward(gout)
    torch.cuda.synchronize(dev)
    vg.grad = None
    Fg.grad = None
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        out = ops.fused_exp_action(None, vg, Fg, L)
        out.backward(gout)
    gr.replay()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    cur = torch.cuda.current_stream(dev)
    e0.record(cur)
    for _ in range(reps):
        gr.replay()
    e1.record(cur)
    torch.cuda.synchronize(dev)
    print(json.dumps({"batch": B, "us_per_step": e0.elapsed_time(e1) * 1e3 / reps}), flush=True)


if __name__ == "__main__":
    main()
