"""Per-layer MIOpen timings of the config-3 conv stacks at batch 512, bf16 NHWC (autocast
layout), forward and backward (dgrad + wgrad via aten.convolution_backward): which
layers dominate the training step.  HIP events over 20 calls each."""
import json
import sys
import torch
sys.path[:0] = ["lie-vae_amd", "."]

dev = torch.device("cuda:0")
torch.backends.cudnn.benchmark = True
B = 512
layers = [  # (name, transposed, Cin, Cout, H_in, stride, pad)
    ("enc1", False, 3, 50, 64, 2, 1), ("enc2", False, 50, 100, 32, 2, 1),
    ("enc3", False, 100, 200, 16, 2, 1), ("enc4", False, 200, 400, 8, 2, 1),
    ("dec2", True, 200, 200, 4, 2, 1), ("dec3", True, 200, 200, 8, 2, 1),
    ("dec4", True, 200, 200, 16, 2, 1), ("dec5", True, 200, 3, 32, 2, 1)]


def timed(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


for name, tr, ci, co, h, st, pd in layers:
    x = torch.randn(B, ci, h, h, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wshape = (ci, co, 4, 4) if tr else (co, ci, 4, 4)
    w = (torch.randn(*wshape, device=dev) * 0.05).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    b = torch.randn(co, device=dev, dtype=torch.bfloat16)
    f = (lambda: torch.nn.functional.conv_transpose2d(x, w, b, st, pd)) if tr else \
        (lambda: torch.nn.functional.conv2d(x, w, b, st, pd))
    y = f()
    gy = torch.randn_like(y)
    bw = lambda: torch.ops.aten.convolution_backward(gy, x, w, [co], [st, st], [pd, pd], [1, 1], tr, [0, 0], 1,  # noqa: E731
                                                     [name != "enc1", True, True])
    ho = y.shape[-1]
    flops = 2.0 * B * ci * co * 16 * (h * h if tr else ho * ho)
    row = {"layer": name, "transposed": tr, "Cin": ci, "Cout": co, "H_in": h, "GFLOP_fwd": flops / 1e9,
           "fwd_us": timed(f), "bwd_us": timed(bw)}
    row["fwd_TFLOPs"] = flops / row["fwd_us"] / 1e6
    print(json.dumps(row), flush=True)
