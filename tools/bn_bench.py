"""Encoder BatchNorm2d + LeakyReLU(0.2), training mode, bf16 channels-last, config-3 shapes
(batch 512): PyTorch's native NHWC BatchNorm (NativeBatchNorm2d below) + leaky_relu vs the
library's fused kernels (nets.FusedBatchNormLeakyReLU), forward and forward+backward, HIP
events over 30 calls.  HBM floor: fwd 3 passes, fwd+bwd 8 passes of the 2·P·C-byte tensor."""
import json
import sys
import torch
sys.path[:0] = ["lie-vae_amd", "."]
from lie_vae.experiments.nets import FusedBatchNormLeakyReLU

dev = torch.device("cuda:0")


class NativeBatchNorm2d(torch.nn.BatchNorm2d):
    """BatchNorm2d by PyTorch's native NHWC kernels (MIOpen disabled for this op only)."""

    def forward(self, x):
        prev = torch.backends.cudnn.enabled
        torch.backends.cudnn.enabled = False
        try:
            return super().forward(x)
        finally:
            torch.backends.cudnn.enabled = prev


def timeit(fn, n=30):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


for (C, H) in [(50, 32), (100, 16), (200, 8), (400, 4)]:
    N = 512
    x = torch.randn(N, C, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    gy = torch.randn_like(x)
    xr = x.clone().requires_grad_(True)
    nat = NativeBatchNorm2d(C).to(dev)
    fus = FusedBatchNormLeakyReLU(C, 0.2).to(dev)
    row = {"N": N, "C": C, "H": H, "MB": x.numel() * 2 / 1e6}
    for tag, mod in (("native", lambda t: torch.nn.functional.leaky_relu(nat(t), 0.2)), ("fused", fus)):
        row[tag + "_fwd_us"] = timeit(lambda: mod(x))
        row[tag + "_fwdbwd_us"] = timeit(lambda: mod(xr).backward(gy))
    row["fused_fwd_TBs"] = 3 * row["MB"] / row["fused_fwd_us"] / 1e6 * 1e6 / 1e6
    row["fused_fwdbwd_TBs"] = 8 * row["MB"] / row["fused_fwdbwd_us"] / 1e6 * 1e6 / 1e6
    print(json.dumps(row), flush=True)
