"""Output fingerprint of the fused forward at config 5 (l = 20, bf16 out) and a ragged batch,
for bitwise A/B of the tile-kernel variants (run once per LV_* knob setting with
LIEVAE_HIP_LIB pointing at the A/B library): prints one JSON line of sha256 digests."""
import hashlib
import json
import os
import sys

import torch

sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lie-vae_amd")]
import lie_vae._ops as ops  # noqa: E402

dev = torch.device("cuda:0")
res = {}
for n, L, dt in ((8192, 20, torch.bfloat16), (1001, 20, torch.bfloat16), (4097, 10, torch.bfloat16),
                 (4096, 10, torch.float32)):
    g = torch.Generator().manual_seed(n + L)
    v = torch.randn(n, 3, generator=g).to(dev)
    F = torch.randn((L + 1) ** 2, 10, generator=g).to(dev)
    out = ops.fused_exp_action(None, v, F, L, out_dtype=dt)
    torch.cuda.synchronize()
    res[f"n{n}_l{L}_{str(dt)[6:]}"] = hashlib.sha256(out.view(torch.int16 if dt == torch.bfloat16 else torch.int32)
                                                     .cpu().numpy().tobytes()).hexdigest()[:16]
print(json.dumps(res), flush=True)
