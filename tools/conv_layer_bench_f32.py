"""Per-layer timings of the config-3 conv stacks at batch 512 in fp32 (the reference's
precision), NCHW and channels-last, MIOpen immediate mode off the packaged find-db (as
the fp32 training step runs): forward, dgrad and wgrad (aten.convolution_backward), plus
fp32 GEMM rates (hipBLASLt via torch.mm) at the sub-pixel GEMM shapes of the 200 -> 200
transposed convolutions.  HIP events over 10 calls each; one JSON line per layer."""
import json
import sys

import torch

sys.path[:0] = ["lie-vae_amd", "."]
from lie_vae.experiments import nets  # noqa: E402

nets.use_packaged_miopen_db()
dev = torch.device("cuda:0")
torch.backends.cudnn.benchmark = False
B = 512
layers = [  # (name, transposed, Cin, Cout, H_in, stride, pad)
    ("enc1", False, 3, 50, 64, 2, 1), ("enc2", False, 50, 100, 32, 2, 1),
    ("enc3", False, 100, 200, 16, 2, 1), ("enc4", False, 200, 400, 8, 2, 1),
    ("dec2", True, 200, 200, 4, 2, 1), ("dec3", True, 200, 200, 8, 2, 1),
    ("dec4", True, 200, 200, 16, 2, 1), ("dec5", True, 200, 3, 32, 2, 1)]


def timed(fn, n=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


tot = {}
for cl in (False, True):
    mf = torch.channels_last if cl else torch.contiguous_format
    for name, tr, ci, co, h, st, pd in layers:
        x = torch.randn(B, ci, h, h, device=dev).contiguous(memory_format=mf)
        wshape = (ci, co, 4, 4) if tr else (co, ci, 4, 4)
        w = (torch.randn(*wshape, device=dev) * 0.05).contiguous(memory_format=mf)
        b = torch.randn(co, device=dev)
        f = (lambda: torch.nn.functional.conv_transpose2d(x, w, b, st, pd)) if tr else \
            (lambda: torch.nn.functional.conv2d(x, w, b, st, pd))
        y = f()
        gy = torch.randn_like(y)
        args = dict(bias_sizes=[co], stride=[st, st], padding=[pd, pd], dilation=[1, 1],
                    transposed=tr, output_padding=[0, 0], groups=1)
        dg = lambda: torch.ops.aten.convolution_backward(gy, x, w, output_mask=[True, False, False], **args)  # noqa
        wg = lambda: torch.ops.aten.convolution_backward(gy, x, w, output_mask=[False, True, True], **args)  # noqa
        r = {"layer": name, "channels_last": cl, "fwd_us": timed(f), "dgrad_us": timed(dg), "wgrad_us": timed(wg)}
        macs = B * y.shape[2] * y.shape[3] * co * ci * (4 if tr else 16)
        r["gflop_per_pass"] = 2 * macs / 1e9
        r["tflops"] = {k: r["gflop_per_pass"] / r[k + "_us"] * 1e-3 for k in ("fwd", "dgrad", "wgrad")}
        print(json.dumps(r), flush=True)
        tot[cl] = tot.get(cl, 0.0) + r["fwd_us"] + r["dgrad_us"] + r["wgrad_us"]
        del x, w, y, gy
print(json.dumps({"total_us_nchw": tot.get(False), "total_us_nhwc": tot.get(True)}), flush=True)
# fp32 GEMM rates at the sub-pixel phase GEMM shapes (M pixels, K = 4 Cin, N = Cout)
for M, K, N in ((512 * 16 * 16, 800, 200), (512 * 8 * 8, 800, 200), (131072, 200, 3200), (200, 131072, 800)):
    a = torch.randn(M, K, device=dev)
    bm = torch.randn(K, N, device=dev)
    us = timed(lambda: torch.mm(a, bm))
    print(json.dumps({"gemm_f32": [M, K, N], "us": us, "tflops": 2 * M * K * N / us / 1e6}), flush=True)
