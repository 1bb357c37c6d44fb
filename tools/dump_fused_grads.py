"""Dump the fused backward's (gmu, gv, gF) and the modular (gang, gF) at one batch size
(same seeded inputs as tests/test_gpu_parity.py::test_shared_spectrum_grads_vs_oracle_fp64)
to gpurun_out/fused_grads_<n>.npz, for analysis against the oracle on the CPU."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lie-vae_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import lie_vae._ops as ops  # noqa: E402
from oracle import lie_ref  # noqa: E402  (input generation only)

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536  # noqa
L, C, M = 10, 10, 121
torch.manual_seed(4242 + n)
gen = torch.Generator().manual_seed(4242 + n)
mu = lie_ref.haar_matrices(n)
v = torch.randn(n, 3, generator=gen) * 0.5
ang = lie_ref.mat_to_eazyz(lie_ref.haar_matrices(n))
F = torch.randn(M, C, generator=gen)
gout = torch.randn(n, M, C, generator=gen)
d = torch.device("cuda:0")
xs = [t.to(d).requires_grad_(True) for t in (mu, v, F)]
(ops.fused_exp_action(*xs, L) * gout.to(d)).sum().backward()
ys = [t.to(d).requires_grad_(True) for t in (mu, v, F)]
import lie_vae.lie_tools as lt  # noqa: E402
z = ops.so3_sample(ys[0], ys[1][None])[0]
angm = lt.group_matrix_to_eazyz(z)
(lt.block_wigner_matrix_multiply(angm, ys[2].expand(n, -1, -1), L) * gout.to(d)).sum().backward()
angf = torch.empty(n, 3, device=d)
os.makedirs("gpurun_out", exist_ok=True)
np.savez(f"gpurun_out/fused_grads_{n}.npz", mu=mu.numpy(), v=v.numpy(), F=F.numpy(), gmu=xs[0].grad.cpu().numpy(), gv=xs[1].grad.cpu().numpy(),
         gF=xs[2].grad.cpu().numpy(), gmu_mod=ys[0].grad.cpu().numpy(), gv_mod=ys[1].grad.cpu().numpy(),
         ang_mod=angm.detach().cpu().numpy())
print("ok", n)
