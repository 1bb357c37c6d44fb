"""Does the fused forward's time depend on the input distribution or on the buffer?
Times lv_fused_exp_action_fwd_repeat (l=10, C=10, fp32) at one batch for v ~ N(0,1),
v ~ U(-1.5, 1.5) and v = 0.1*N(0,1), each into a fresh and into a reused output."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lie-vae_amd"))
from lie_vae import _lib  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    L, C = 10, 10
    M = (L + 1) ** 2
    F = torch.randn(M, C, device=dev)
    out = torch.empty(n, M, C, device=dev)
    s = torch.cuda.current_stream()
    sp = ctypes.c_void_p(s.cuda_stream)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    res = {}
    for name, v in (("randn", torch.randn(n, 3, device=dev)),
                    ("uniform1.5", (torch.rand(n, 3, device=dev) - 0.5) * 3),
                    ("small", 0.1 * torch.randn(n, 3, device=dev))):
        for reps in (50, 200):
            for _ in range(2):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                rc = lib.lv_fused_exp_action_fwd_repeat(None, P(v), P(F), 0, P(out), 0, None, n, L,
                                                        C, 0, reps, sp)
                assert rc == 0, _lib.last_error()
                e1.record(s)
                torch.cuda.synchronize()
            res[f"{name}_x{reps}"] = e0.elapsed_time(e1) * 1e3 / reps
    print(json.dumps({"n": n, "us_per_launch": res}), flush=True)


if __name__ == "__main__":
    main()
