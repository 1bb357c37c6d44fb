"""Start gate for the short timed region: the GPU waits (hipStreamWaitValue32 on a
coherent pinned-host flag) until the host has submitted the events and the whole graph,
so ev0 -> ev1 times the kernels, not the host's graph submission.  Compared against
stream events around an ungated replay (K = 20) and a long run (K = 100 x 5)."""
import ctypes
import sys
import threading
import torch
sys.path[:0] = ["lie-vae_amd", "."]
from lie_vae import _lib

hip = ctypes.CDLL("libamdhip64.so")
hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
hip.hipStreamWaitValue32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint,
                                     ctypes.c_uint32]
dev = torch.device("cuda:0")
lib = _lib.load()
B, L, C = 4096, 10, 10
v = torch.randn(B, 3, device=dev)
F = torch.randn(121, C, device=dev)
out = torch.empty(B, 121, C, device=dev)
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
cur = torch.cuda.current_stream()


def launch(k, s):
    assert lib.lv_fused_exp_action_fwd_repeat(None, P(v), P(F), 0, P(out), 0, None, B, L, C, 0, k,
                                              ctypes.c_void_p(s.cuda_stream)) == 0


flag = ctypes.c_void_p()
rc = hip.hipHostMalloc(ctypes.byref(flag), 64, 0x40000000)  # hipHostMallocCoherent
print("hipHostMalloc rc", rc)
fv = ctypes.cast(flag, ctypes.POINTER(ctypes.c_uint32))
launch(5, cur)
torch.cuda.synchronize()
graphs = {}
for K in (20, 100):
    s = torch.cuda.Stream()
    s.wait_stream(cur)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        launch(K, s)
    g.replay()
    torch.cuda.synchronize()
    graphs[K] = g
for rep in range(3):
    for gated in (False, True):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fv[0] = 0
        torch.cuda.synchronize()
        guard = None
        if gated:
            r = hip.hipStreamWaitValue32(ctypes.c_void_p(cur.cuda_stream), flag, 1, 0, 0xFFFFFFFF)
            if r != 0:
                print("hipStreamWaitValue32 rc", r)
                fv[0] = 1
                continue
            guard = threading.Timer(2.0, lambda: fv.__setitem__(0, 1))  # never leave it waiting
            guard.start()
        try:
            e0.record(cur)
            graphs[20].replay()
            e1.record(cur)
        finally:
            fv[0] = 1
        torch.cuda.synchronize()
        if guard:
            guard.cancel()
        print(f"rep {rep} gated={gated}: K=20 {e0.elapsed_time(e1) * 1e3 / 20:.3f} us/launch")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(cur)
    for _ in range(5):
        graphs[100].replay()
    e1.record(cur)
    torch.cuda.synchronize()
    print(f"rep {rep}: K=500 {e0.elapsed_time(e1) * 1e3 / 500:.3f} us/launch")
