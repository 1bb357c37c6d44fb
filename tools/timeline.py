"""Phase timeline of the group-action tile kernels from in-kernel timestamps (A/B build,
LV_STAMPS=1: lane 0 of every wave writes the 100 MHz real-time counter at each phase
boundary; action_common.h phase_stamp).  For the last of R back-to-back launches of the
fused forward and of lv_group_action_bwd at one shape, prints per degree segment (wave
index) the median / 90th-percentile phase durations and, over the whole grid, when blocks
start / finish relative to the earliest block start (10 ns ticks shown as us).

  LIEVAE_HIP_LIB=lie-vae_amd/lie_vae/liblievae_hip_ab.so LV_STAMPS=1 \
      python tools/timeline.py [B] [L] [f32|bf16] [fwd|bwd|both]
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lie-vae_amd")]
from lie_vae import _lib  # noqa: E402

KB = 16384  # kStampBlocks
TICK_US = 0.01  # s_memrealtime: 100 MHz


DEG_BASE, DEG_BLOCKS = KB * 16 * 8 + 2 * 4096, 2048


def stamps(lib, with_deg=False):
    n = DEG_BASE + DEG_BLOCKS * 16 * 24
    buf = np.zeros(n, dtype=np.uint64)
    fn = lib.lv_ab_stamps_copy
    fn.restype, fn.argtypes = ctypes.c_size_t, [ctypes.c_void_p, ctypes.c_size_t]
    got = fn(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes))
    assert got == buf.nbytes, "LV_STAMPS=1 and the A/B library (LIEVAE_HIP_LIB) are required"
    out = (buf[: KB * 16 * 8].reshape(KB, 16, 8).astype(np.int64),
           buf[KB * 16 * 8: DEG_BASE].reshape(4096, 2).astype(np.int64))
    if with_deg:
        out = out + (buf[DEG_BASE:].reshape(DEG_BLOCKS, 16, 24).astype(np.int64),)
    return out


def degree_costs(name, st, deg, nblk, masks):
    """Median time per degree (us): stamp at the end of degree l minus the end of the
    wave's previous degree (phase-1 stamp for its first), in the order the wave ran them
    (the backward walks its degrees largest first, the forward smallest first)."""
    nb = min(nblk, DEG_BLOCKS)
    res = {}
    for w, m in enumerate(masks):
        prev = st[:nb, w, 1]
        ls = [b for b in range(24) if (m >> b) & 1]
        ls.sort(key=lambda b: float(np.median(deg[:nb, w, b])))  # execution order
        for l in ls:
            d = (deg[:nb, w, l] - prev) * TICK_US
            res[l] = (w, float(np.median(d)))
            prev = deg[:nb, w, l]
    print(f"  {name} per-degree median us: " + " ".join(f"l{l}(w{w}):{t:.3f}" for l, (w, t) in sorted(res.items())))
    return res


def report(name, st, nblk, nwave, phases, red=None, nred=0, extra=None):
    s = st[:nblk, :nwave, :]
    t0 = s[:, :, 0][s[:, :, 0] > 0].min()
    print(f"== {name}: {nblk} blocks x {nwave} waves")
    us = lambda x: x * TICK_US  # noqa: E731
    for w in range(nwave):
        cols = []
        for k in range(1, len(phases)):
            d = us(s[:, w, k] - s[:, w, k - 1])
            cols.append(f"{phases[k]} {np.median(d):6.2f}/{np.percentile(d, 90):6.2f}")
        print(f"  wave {w}: " + "  ".join(cols))
    start = us(s[:, 0, 0] - t0)
    end = us(s[:, :, len(phases) - 1].max(axis=1) - t0)
    print(f"  block start  p10/50/90/max {np.percentile(start, 10):6.2f} {np.median(start):6.2f} "
          f"{np.percentile(start, 90):6.2f} {start.max():6.2f} us")
    print(f"  block finish p10/50/90/max {np.percentile(end, 10):6.2f} {np.median(end):6.2f} "
          f"{np.percentile(end, 90):6.2f} {end.max():6.2f} us")
    if extra:
        for k, nm in extra:
            d = us(s[:, :, k] - s[:, :, 0])
            ok = s[:, :, k] > 0
            print(f"  {nm}: median " + " ".join(f"{np.median(d[:, w][ok[:, w]]):5.2f}" if ok[:, w].any() else "  -  "
                                            for w in range(nwave)) + " us after wave start")
    first = [us(np.median(s[:, w, 1] - t0)) for w in range(nwave)]
    print("  median time of phase 1 end per wave (from grid start): " + " ".join(f"{x:5.2f}" for x in first))
    if red is not None and nred:
        r = red[:nred]
        print(f"  reduce kernel: start p50 {us(np.median(r[:, 0] - t0)):6.2f}  end max {us(r[:, 1].max() - t0):6.2f} us"
              f"  (tile grid finished at {end.max():6.2f})")


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    L = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    dt = sys.argv[3] if len(sys.argv) > 3 else "f32"
    which = sys.argv[4] if len(sys.argv) > 4 else "both"
    C, R = 10, 30
    dev = torch.device("cuda:0")
    lib = _lib.load()
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    g = torch.Generator().manual_seed(0)
    v = torch.randn(B, 3, generator=g).to(dev)
    M = (L + 1) ** 2
    F = torch.randn(M, C, generator=g).to(dev)
    odt = torch.bfloat16 if dt == "bf16" else torch.float32
    out = torch.empty(B, M, C, device=dev, dtype=odt)
    ang = torch.empty(B, 3, device=dev)
    plan = (ctypes.c_int64 * 40)()
    code = _lib.LV_DTYPE_BF16 if dt == "bf16" else _lib.LV_DTYPE_F32
    assert lib.lv_action_fwd_plan(1, 0, code, B, L, C, plan) == 0
    if which in ("fwd", "both"):
        for _ in range(R):
            assert lib.lv_fused_exp_action_fwd(None, P(v), P(F), 0, P(out), code, P(ang), B, L, C, 0, None) == 0
        st, _, deg = stamps(lib, True)
        print(f"plan: blocks {plan[1]} segments {plan[2]} lds {plan[4]} degree sets "
              f"{[bin(plan[24 + k]) for k in range(plan[2])]}")
        report(f"fused forward B={B} l={L} {dt}", st, min(plan[1], KB), plan[2],
               ["start", "prologue", "chain", "barrier", "flush"],
               extra=[(5, "loads landed"), (6, "exp->ZYZ done (wave 0)"), (7, "multiples done (wave 0)")])
        degree_costs("forward", st, deg, plan[1], [plan[24 + k] for k in range(plan[2])])
    if which in ("bwd", "both"):
        lib.lv_fused_exp_action_fwd(None, P(v), P(F), 0, P(out), _lib.LV_DTYPE_F32, P(ang), B, L, C, 0, None)
        gout = torch.randn(B, M, C, generator=g).to(dev)
        gang, gF = torch.empty(B, 3, device=dev), torch.empty(M, C, device=dev)
        wsb = lib.lv_group_action_bwd_workspace(B, L, C, 1)
        ws = torch.zeros(max(wsb, 1), device=dev, dtype=torch.uint8)
        bp = (ctypes.c_int64 * 40)()
        assert lib.lv_group_action_bwd_plan(B, L, C, 1, bp) == 0
        for _ in range(R):
            assert lib.lv_group_action_bwd(P(ang), P(F), 0, P(gout), P(gang), P(gF), B, L, C, 0, P(ws), wsb,
                                           None) == 0
        st, red, deg = stamps(lib, True)
        print(f"bwd plan: blocks {bp[1]} segments {bp[2]} lds {bp[4]} degree sets {[bin(bp[24 + k]) for k in range(bp[2])]}")
        report(f"group-action backward B={B} l={L}", st, min(bp[1], KB), bp[2],
               ["start", "load+prologue", "chain", "slab", "angle-sync", "end"], red, (M * C + 15) // 16)
        degree_costs("backward", st, deg, bp[1], [bp[24 + k] for k in range(bp[2])])


if __name__ == "__main__":
    main()
