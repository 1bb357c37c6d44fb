"""Decoder ConvTranspose2d(200, 200, 4, 2, 1) forward at the config-3 batch (512), bf16
NHWC: MIOpen (torch conv_transpose2d) vs the library's MFMA kernels (lv_deconv4s2_fwd_bf16,
pack + GEMM; v1 at 128 / 256 pixel rows, v2 with a 2 / 3-stage LDS-DMA ring), HIP events
over 50 calls each, v2 output bit-compared with v1.  FLOPs = 2 * N * Cin * Cout * 16 * H * W."""
import json
import sys
import torch
sys.path[:0] = ["lie-vae_amd", "."]
from lie_vae.experiments.nets import _Deconv4s2

dev = torch.device("cuda:0")
torch.backends.cudnn.benchmark = True
res = []
for (N, C, H) in [(512, 200, 4), (512, 200, 8), (512, 200, 16), (512, 3, 32)]:
    Ci, Co = 200, C
    x = torch.randn(N, Ci, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Ci, Co, 4, 4, device=dev) * 0.05).to(torch.bfloat16)
    b = torch.randn(Co, device=dev)
    wcl = w.contiguous(memory_format=torch.channels_last)
    flops = 2.0 * N * Ci * Co * 16 * H * H
    row = {"N": N, "Cin": Ci, "Cout": Co, "H_in": H, "GFLOP": flops / 1e9}
    from lie_vae import _lib
    big = Co % 8 == 0
    if big:
        wt = torch.empty(_lib.load().lv_deconv4s2_packed_weight_elems(Ci), device=dev, dtype=torch.bfloat16)
        _lib.call("lv_deconv4s2_pack_weight_bf16", w.data_ptr(), wt.data_ptr(), Ci, Co, _lib.stream())
    yk = torch.empty(N, Co, 2 * H, 2 * H, device=dev, dtype=torch.bfloat16, memory_format=torch.channels_last)

    def kern(bm):
        _lib.call("lv_deconv4s2_fwd_bf16_tile", x.data_ptr(), wt.data_ptr(), b.data_ptr(), yk.data_ptr(),
                  N, H, H, Ci, Co, bm, _lib.stream())
    runs = [("miopen", lambda: torch.nn.functional.conv_transpose2d(x, wcl, b.to(torch.bfloat16), 2, 1)),
            ("mfma", lambda: _Deconv4s2.apply(x, w, b))]
    if big:
        runs += [("gemm_bm128", lambda: kern(128)), ("gemm_bm256", lambda: kern(256)),
                 ("v2_s2", lambda: kern(2)), ("v2_s3", lambda: kern(3)),
                 ("v2_s2_xcd", lambda: kern(4)), ("v2_s3_xcd", lambda: kern(5)),
                 ("v2_128_s2_xcd", lambda: kern(6)), ("v2_128_s3_xcd", lambda: kern(7)),
                 ("v2_128_s2_xcd_rm", lambda: kern(8)), ("v2_128_s2_xcd_b", lambda: kern(6)),
                 ("v2_128_s2_xcd_rm_b", lambda: kern(8))]
    for tag, fn in runs:
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 50
        row[tag + "_us"] = us
        row[tag + "_TFLOPs"] = flops / us / 1e6
    if big:  # v2 (both ring depths) against v1: the same MFMA sequence per element
        kern(256)
        y1 = yk.clone()
        for v in (2, 3, 4, 5, 6, 7, 8):
            yk.fill_(float("nan"))
            kern(v)
            row[f"v2_{v}_bitwise_vs_v1"] = bool(torch.equal(yk, y1))
    ref = torch.nn.functional.conv_transpose2d(x.float(), w.float(), b, 2, 1)
    y = _Deconv4s2.apply(x, w, b).float()
    row["max_rel_err_vs_f32"] = float(((y - ref).abs().max() / ref.abs().max()).item())
    res.append(row)
    print(json.dumps(row), flush=True)
