"""fp32 decoder layers at batch 512 (config 3's fp32 step): ConvTranspose2d(200, 200, 4, 2, 1)
at 4 -> 8, 8 -> 16, 16 -> 32 -- torch's fp32 layer (MIOpen, NCHW, packaged find-db) against
lv_deconv4s2_fwd_f32 (fp32 MFMA): the kernel alone (channels-last input, packed weight) and
the module path (_Deconv4s2F32.forward: weight pack + channels-last copy + kernel).  HIP
events over 10 calls each; one JSON line per layer, with the max error of each against a
float64 evaluation of one image."""
import json
import sys

import torch

sys.path[:0] = ["lie-vae_amd", "."]
from lie_vae import _lib  # noqa: E402
from lie_vae.experiments import nets  # noqa: E402

nets.use_packaged_miopen_db()
dev = torch.device("cuda:0")
torch.backends.cudnn.benchmark = False
B = 512


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


# argv[1] (optional): one input size only, e.g. 16 for the 16 -> 32 layer (PMC runs)
for H in ((int(sys.argv[1]),) if len(sys.argv) > 1 else (4, 8, 16)):
    Cin = Cout = 200
    g = torch.Generator(device=dev).manual_seed(H)
    x = torch.randn(B, Cin, H, H, device=dev, generator=g)
    w = torch.randn(Cin, Cout, 4, 4, device=dev, generator=g) * 0.05
    b = torch.randn(Cout, device=dev, generator=g)
    xc = x.contiguous(memory_format=torch.channels_last)
    wt = torch.empty(_lib.load().lv_deconv4s2_packed_weight_elems_f32(Cin), device=dev)
    st = _lib.stream()
    _lib.call("lv_deconv4s2_pack_weight_f32", w.data_ptr(), wt.data_ptr(), Cin, Cout, st)
    y = torch.empty(B, Cout, 2 * H, 2 * H, device=dev)

    def kern():
        _lib.call("lv_deconv4s2_fwd_f32", xc.data_ptr(), wt.data_ptr(), b.data_ptr(), y.data_ptr(), None,
                  B, H, H, Cin, Cout, 0, st)
    t_m = timed(lambda: torch.nn.functional.conv_transpose2d(x, w, b, 2, 1))
    t_k = timed(kern)
    t_p = timed(lambda: nets._Deconv4s2F32.apply(x, w, b, 0)[0])
    yt = torch.nn.functional.conv_transpose2d(x, w, b, 2, 1)
    kern()
    torch.cuda.synchronize()
    ref = torch.nn.functional.conv_transpose2d(x[:1].double(), w.double(), b.double(), 2, 1)
    gflop = 2 * B * (2 * H) ** 2 * Cout * Cin * 4 / 1e9
    print(json.dumps({"layer": f"{H}->{2 * H}", "gflop": gflop, "miopen_us": t_m, "mfma_f32_kernel_us": t_k,
                      "mfma_f32_path_us": t_p, "miopen_tflops": gflop / t_m * 1e-3,
                      "mfma_f32_tflops": gflop / t_k * 1e-3,
                      "err_miopen": (yt[:1].double() - ref).abs().max().item(),
                      "err_mfma_f32": (y[:1].double() - ref).abs().max().item(),
                      "max_diff_full_batch": (y - yt).abs().max().item()}), flush=True)
