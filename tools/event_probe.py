"""Does a torch.cuda.Event recorded during hipGraph capture time the graph's kernels on
ROCm?  Captures [ev0, K fused-forward launches, ev1] and compares ev0->ev1 against
events recorded on the stream around graph.replay()."""
import ctypes
import sys
import torch
sys.path[:0] = ["lie-vae_amd", "."]
from lie_vae import _lib

dev = torch.device("cuda:0")
lib = _lib.load()
B, L, C = 4096, 10, 10
v = torch.randn(B, 3, device=dev)
F = torch.randn(121, C, device=dev)
out = torch.empty(B, 121, C, device=dev)
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731


def launch(k, s):
    assert lib.lv_fused_exp_action_fwd_repeat(None, P(v), P(F), 0, P(out), 0, None, B, L, C, 0, k,
                                              ctypes.c_void_p(s.cuda_stream)) == 0


cur = torch.cuda.current_stream()
launch(5, cur)
torch.cuda.synchronize()
for K in (20, 100):
    s = torch.cuda.Stream()
    s.wait_stream(cur)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(g, stream=s):
            e0.record(s)
            launch(K, s)
            e1.record(s)
    except Exception as ex:  # noqa: BLE001
        print("capture with events failed:", repr(ex))
        continue
    g.replay()
    torch.cuda.synchronize()
    for rep in range(3):
        o0, o1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        o0.record(cur)
        g.replay()
        o1.record(cur)
        torch.cuda.synchronize()
        try:
            ig = e0.elapsed_time(e1) * 1e3 / K
        except Exception as ex:  # noqa: BLE001
            ig = repr(ex)
        print(f"K={K} rep={rep}: stream events {o0.elapsed_time(o1) * 1e3 / K:.3f} us/launch, "
              f"in-graph events {ig}")
