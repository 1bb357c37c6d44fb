"""SO(3) tools — drop-in for ``lie_vae.lie_tools`` (reference ``lie_vae/lie_tools.py``).

Same names, argument meaning and shape asserts as the reference; the numerical work
runs in the HIP kernels of ``liblievae_hip.so`` (fp32; the Gram–Schmidt map in fp64 as
in the reference).  Inputs must live on a HIP device — there is no CPU fallback.
Pure data rearrangements (hat/vee) and the RNG-driven samplers stay tensor ops on
whatever device the caller uses.
"""
import math
from functools import lru_cache

import numpy as np
import torch

from . import _ops
from ._jtab import j_numpy

__all__ = [
    "j_matrix", "map_to_lie_algebra", "map_to_lie_vector", "rodrigues", "s2s1rodrigues",
    "s2s2_gram_schmidt", "vector_to_eazyz", "log_map", "group_matrix_to_quaternions",
    "quaternions_to_eazyz", "group_matrix_to_eazyz", "quaternions_to_group_matrix",
    "wigner_d_matrix", "block_wigner_matrix_multiply", "random_quaternions",
    "random_group_matrices",
]


@lru_cache(maxsize=256)
def j_matrix(l, device=None):
    """J_l (fp32) — reference lie_tools.py:10-14 (lie_learn Jd, regenerated here)."""
    return torch.tensor(j_numpy(l), dtype=torch.float32, device=torch.device(device or "cpu"))


def map_to_lie_algebra(v):
    """hat: (...,3) -> (...,3,3) — lie_tools.py:17-43."""
    assert v.size()[-1] == 3
    z = torch.zeros_like(v[..., 0])
    x, y, w = v[..., 0], v[..., 1], v[..., 2]
    return torch.stack([z, -w, y, w, z, -x, -y, x, z], -1).reshape(*v.shape[:-1], 3, 3)


def map_to_lie_vector(X):
    """vee — lie_tools.py:46-53."""
    return torch.stack((-X[..., 1, 2], X[..., 0, 2], -X[..., 0, 1]), -1)


def rodrigues(v):
    """so(3) exp, (...,3) -> (...,3,3) — lie_tools.py:56-64 (NaN at |v| = 0, as there)."""
    assert v.shape[-1] == 3
    return _ops.unary(v, _ops.SO3_EXP)


def s2s1rodrigues(s2_el, s1_el):
    """lie_tools.py:67-78."""
    return _ops.s2s1(s2_el, s1_el)


def s2s2_gram_schmidt(v1, v2):
    """lie_tools.py:81-89, fp64 like S2S2Mean (cross along the last axis)."""
    out = _ops.s2s2(v1, v2)
    return out if v1.dtype == torch.float64 else out.to(v1.dtype)


def vector_to_eazyz(v):
    """tanh squashing to ZYZ ranges — lie_tools.py:92-97 (latent modes normal/vmf)."""
    angles = torch.tanh(v) * v.new_tensor([math.pi, math.pi / 2, math.pi])
    return angles + v.new_tensor([0, math.pi / 2, 0])


def log_map(R):
    """Unbatched log map (reference test helper) — lie_tools.py:100-109."""
    anti_sym = .5 * (R - R.transpose(-1, -2))
    theta = torch.acos(.5 * (torch.trace(R) - 1))
    return theta / torch.sin(theta) * anti_sym


def group_matrix_to_quaternions(r):
    """Scalar-last quaternions — lie_tools.py:112-157."""
    assert list(r.shape[-2:]) == [3, 3], 'Input must be 3x3 matrices'
    return _ops.unary(r, _ops.MAT_TO_QUAT)


def quaternions_to_eazyz(q):
    """ZYZ Euler angles, not mod 2π — lie_tools.py:160-175."""
    assert q.shape[-1] == 4, 'Input must be 4 dim vectors'
    return _ops.unary(q, _ops.QUAT_TO_EAZYZ)


def group_matrix_to_eazyz(r):
    """lie_tools.py:178-180 (one fused kernel)."""
    assert list(r.shape[-2:]) == [3, 3], 'Input must be 3x3 matrices'
    return _ops.unary(r, _ops.MAT_TO_EAZYZ)


def quaternions_to_group_matrix(q):
    """Normalises q — lie_tools.py:183-192."""
    assert q.shape[-1] == 4
    return _ops.unary(q, _ops.QUAT_TO_MAT)


def wigner_d_matrix(angles, degree):
    """D_l(α,β,γ) = X(α)·J·X(β)·J·X(γ), (...,3) -> (...,2l+1,2l+1) — lie_tools.py:211-223.

    Materialises D (debug / parity use); the decoder path never does."""
    assert angles.shape[-1] == 3, 'Input must be 3 dim vectors'
    lead = angles.shape[:-1]
    a = angles.reshape(-1, 3)
    n = 2 * degree + 1
    D = _ops.wigner_blocks(a, degree)
    off = degree * (2 * degree - 1) * (2 * degree + 1) // 3
    return D[:, off:off + n * n].reshape(*lead, n, n)


def block_wigner_matrix_multiply(angles, spectrum, max_degree, transpose=False):
    """Block-diagonal D(g)·F for l = 0..max_degree — lie_tools.py:226-253.

    angles (batch, 3); spectrum (batch, (L+1)^2, C), a stride-0 expand of a
    ((L+1)^2, C) tensor (shared, as ActionNet passes it) or a per-sample tensor.
    Output (batch, (L+1)^2, C)."""
    return _ops.group_action(angles, spectrum, max_degree, transpose=transpose)


def random_quaternions(n, dtype=torch.float32, device=None):
    """Haar-uniform quaternions (Shoemake) — lie_tools.py:256-263."""
    u1, u2, u3 = torch.rand(3, n, dtype=dtype, device=device)
    return torch.stack((
        torch.sqrt(1 - u1) * torch.sin(2 * np.pi * u2),
        torch.sqrt(1 - u1) * torch.cos(2 * np.pi * u2),
        torch.sqrt(u1) * torch.sin(2 * np.pi * u3),
        torch.sqrt(u1) * torch.cos(2 * np.pi * u3),
    ), 1)


def random_group_matrices(n, dtype=torch.float32, device=None):
    """lie_tools.py:266-267."""
    return quaternions_to_group_matrix(random_quaternions(n, dtype, device))
