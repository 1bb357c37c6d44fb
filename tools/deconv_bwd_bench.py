"""Decoder ConvTranspose2d(200, Cout, 4, 2, 1) BACKWARD at the config-3 batch (512), bf16
NHWC, HIP events over 30 calls each:
  miopen  aten.convolution_backward (gx, gw, gb) -- what the plain layer runs
  lib     _Deconv4s2.backward: Cout <= 4 -> lv_deconv4s2_small_bwd_bf16 (dgrad + wgrad +
          bias); else MIOpen gx/gw without bias + lv_channel_sum_bf16
  parts   the library's dgrad-only / wgrad-only calls (small) and the bias sum alone.
HBM floor: gx write + x read = 2 * 2 * N * H * W * Cin bytes (+ gy), reported as GB/s."""
import json
import sys
import torch
sys.path[:0] = ["lie-vae_amd", "."]
from lie_vae import _lib
from lie_vae.experiments.nets import _Deconv4s2, _channel_sum

dev = torch.device("cuda:0")
torch.backends.cudnn.benchmark = True


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


for (N, Co, H) in [(512, 3, 32), (512, 200, 16), (512, 200, 8)]:
    Ci = 200
    x = torch.randn(N, Ci, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Ci, Co, 4, 4, device=dev) * 0.05).to(torch.bfloat16)
    b = torch.randn(Co, device=dev)
    gy = torch.randn(N, Co, 2 * H, 2 * H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    row = {"N": N, "Cin": Ci, "Cout": Co, "H_in": H}
    row["miopen_us"] = timeit(lambda: torch.ops.aten.convolution_backward(
        gy, x, w, [Co], [2, 2], [1, 1], [1, 1], True, [0, 0], 1, [True, True, True]))

    class Ctx:
        saved_tensors = (x, w)
        has_bias = True
        needs_input_grad = (True, True, True)
    row["lib_us"] = timeit(lambda: _Deconv4s2.backward(Ctx, gy))
    row["bias_sum_us"] = timeit(lambda: _channel_sum(gy)) if Co % 8 == 0 else None
    if Co <= 4:
        lib, st = _lib.load(), _lib.stream()
        wd = torch.empty(lib.lv_deconv4s2_small_dgrad_weight_elems(Ci), device=dev, dtype=torch.bfloat16)
        _lib.call("lv_deconv4s2_small_pack_dgrad_weight_bf16", w.data_ptr(), wd.data_ptr(), Ci, Co, st)
        gx = torch.empty_like(x)
        gw = torch.empty_like(w)
        gb = torch.empty(Co, device=dev)
        ws = torch.empty(lib.lv_deconv4s2_small_bwd_workspace_elems(N, H, H, Ci, Co), device=dev)
        row["dgrad_us"] = timeit(lambda: _lib.call("lv_deconv4s2_small_bwd_bf16", x.data_ptr(), gy.data_ptr(),
                                                   wd.data_ptr(), gx.data_ptr(), None, None, None, N, H, H, Ci, Co, st))
        row["wgrad_us"] = timeit(lambda: _lib.call("lv_deconv4s2_small_bwd_bf16", x.data_ptr(), gy.data_ptr(),
                                                   None, None, gw.data_ptr(), gb.data_ptr(), ws.data_ptr(),
                                                   N, H, H, Ci, Co, st))
        act = 2.0 * N * H * H * Ci
        row["dgrad_GBs"] = act / row["dgrad_us"] / 1e3
        row["wgrad_GBs"] = act / row["wgrad_us"] / 1e3
    print(json.dumps(row), flush=True)
