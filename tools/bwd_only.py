#!/usr/bin/env python3
"""Backward-only, graph-replayed lv_group_action_bwd (tile kernel + dF reduce) at one
batch, for a rocprofv3 kernel trace that reconciles with bench.py's fwd_bwd.action_bwd
figure (same call, same capture: 50 calls per graph, replayed).

  rocprofv3 --kernel-trace --stats -d gpurun_out/p -o run -- python3 tools/bwd_only.py 4096

Third argument "fused": lv_fused_exp_action_bwd instead (the training path: the same
kernels plus the exp -> ZYZ VJP, v -> gv, from the forward's saved angles).
"""
import ctypes
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "lie-vae_amd"), REPO]


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    fused = len(sys.argv) > 3 and sys.argv[3] == "fused"
    L, C = 10, 10
    M = (L + 1) ** 2
    from lie_vae import _lib
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(7)
    ang = (torch.rand(B, 3, generator=g) * 6 - 3).to(dev)
    F = torch.randn(M, C, generator=g).to(dev)
    gout = torch.randn(B, M, C, generator=g).to(dev)
    gang = torch.empty(B, 3, device=dev)
    gF = torch.empty(M, C, device=dev)
    ws_bytes = lib.lv_group_action_bwd_workspace(B, L, C, 1)
    ws = torch.empty(max(ws_bytes, 1), device=dev, dtype=torch.uint8)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    s = torch.cuda.Stream(dev)

    v = (torch.rand(B, 3, generator=g) * 2 - 1).to(dev)
    gv = torch.empty(B, 3, device=dev)
    if fused:  # the forward's saved angles for v
        out = torch.empty(B, (L + 1) ** 2, C, device=dev)
        rc = lib.lv_fused_exp_action_fwd(None, P(v), P(F), 0, P(out), 0, P(ang), B, L, C, 0,
                                         ctypes.c_void_p(s.cuda_stream))
        if rc:
            raise RuntimeError(_lib.last_error())
        torch.cuda.synchronize(dev)

    def call(k):
        for _ in range(k):
            if fused:
                rc = lib.lv_fused_exp_action_bwd(None, P(v), P(ang), P(F), P(gout), None, P(gv), P(gF),
                                                 B, L, C, 0, P(ws), ws_bytes, ctypes.c_void_p(s.cuda_stream))
            else:
                rc = lib.lv_group_action_bwd(P(ang), P(F), 0, P(gout), P(gang), P(gF), B, L, C, 0,
                                             P(ws), ws_bytes, ctypes.c_void_p(s.cuda_stream))
            if rc:
                raise RuntimeError(_lib.last_error())

    with torch.cuda.stream(s):
        call(2)
    torch.cuda.synchronize(dev)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=s):
        call(50)
    gr.replay()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    cur = torch.cuda.current_stream(dev)
    e0.record(cur)
    for _ in range(reps):
        gr.replay()
    e1.record(cur)
    torch.cuda.synchronize(dev)
    us = e0.elapsed_time(e1) * 1e3 / (reps * 50)
    import hashlib
    import numpy as np
    gf = gF.cpu().numpy()
    np.save(os.path.join(REPO, "gpurun_out", f"bwd_only_gF_{B}_{os.environ.get('LV_BWD_VARIANT', 'd')}.npy"), gf)
    print(json.dumps({"batch": B, "fused": fused, "calls": reps * 50, "us_per_call": us,
                      "gF_sha": hashlib.sha1(gf.tobytes()).hexdigest()[:12],
                      "gang_sha": hashlib.sha1(gang.cpu().numpy().tobytes()).hexdigest()[:12],
                      "plan": _lib.plan("bwd", B, L, C, 1)}), flush=True)


if __name__ == "__main__":
    main()
