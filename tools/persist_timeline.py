#!/usr/bin/env python3
"""Phase timeline of the persistent backward (A/B build, LV_STAMPS=1): stamps of each
block's 5th group at 8 phase boundaries (action_bwd_persist.h st(k, ph)); prints the median
duration of each phase per wave over blocks.  100 MHz real-time counter (10 ns ticks).
  LIEVAE_HIP_LIB=.../liblievae_hip_ab.so LV_STAMPS=1 python tools/persist_timeline.py 65536"""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "lie-vae_amd"), REPO]


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    L, C = 10, 10
    M = (L + 1) ** 2
    from lie_vae import _lib
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    ang = (torch.rand(B, 3) * 6 - 3).to(dev)
    F = torch.randn(M, C).to(dev)
    gout = torch.randn(B, M, C).to(dev)
    gang = torch.empty(B, 3, device=dev)
    gF = torch.empty(M, C, device=dev)
    wsb = lib.lv_group_action_bwd_workspace(B, L, C, 1)
    ws = torch.empty(wsb, device=dev, dtype=torch.uint8)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    for _ in range(3):
        rc = lib.lv_group_action_bwd(P(ang), P(F), 0, P(gout), P(gang), P(gF), B, L, C, 0, P(ws), wsb, None)
        assert rc == 0, _lib.last_error()
    torch.cuda.synchronize()
    f = lib.lv_ab_stamps_copy
    f.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    f.restype = ctypes.c_size_t
    nblk = _lib.plan("bwd", B, L, C, 1)["blocks"]
    buf = np.zeros(16384 * 16 * 8, dtype=np.uint64)
    got = f(buf.ctypes.data, buf.nbytes)
    st = buf[: nblk * 16 * 8].reshape(nblk, 16, 8).astype(np.int64)
    names = ["chain", "slab pass", "partials", "barrier B", "DMA issue+gang sums+fill", "tile DMA wait", "barrier A"]
    print(f"persistent backward B={B}: {nblk} blocks, phase durations of the 5th group (median / p90 us)")
    for w in range(4):
        s = st[:, w, :]
        ok = (s[:, 0] > 0) & (s[:, 7] > 0)
        d = np.diff(s[ok], axis=1) * 0.01  # 100 MHz -> us
        row = "  ".join(f"{n} {np.median(d[:, i]):.2f}/{np.percentile(d[:, i], 90):.2f}" for i, n in enumerate(names))
        print(f"  wave {w}: {row}  (n={ok.sum()})")
    tot = (st[:, 0, 7] - st[:, 0, 0]) * 0.01
    tot = tot[tot > 0]
    print(f"  group total (wave 0): median {np.median(tot):.2f} us")


if __name__ == "__main__":
    main()
