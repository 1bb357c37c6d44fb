"""Latent reparameterisers — drop-in for ``lie_vae.reparameterize``.

Same module names, constructor arguments, stateful attributes (``sigma``, ``z``,
``mu_lie``, ``v``) and methods (``forward(x, n)``, ``kl``, ``log_posterior``,
``log_prior``, ``nsample``, ``deterministic``) as reference
``lie_vae/reparameterize.py``.  The SO(3) maths runs in HIP kernels:

* softplus σ and v = ε·σ                 (N0reparameterize, :100-145)
* z = μ·exp(v)                            (SO3reparameterize.nsample, :269-273)
* 21-term wrapped log-density + logsumexp (SO3reparameterize.log_posterior, :233-263)
* mean maps rodrigues / quaternion / S2S1 / fp64 S2S2 (:148-197)

Extension (superset of the reference API): ``forward(x, n, eps=None)`` accepts an
injected standard-normal ε of shape (n, B, z_dim), used by the parity tests; by
default ε is drawn on the device with ``torch.randn`` as the reference's
``Normal.sample`` does.
"""
import math

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.distributions import Normal

from . import _ops
from .lie_tools import (quaternions_to_group_matrix, rodrigues, s2s1rodrigues,
                        s2s2_gram_schmidt)


class Nreparameterize(nn.Module):
    """Euclidean Gaussian latent (baseline mode) — reparameterize.py:16-55."""

    def __init__(self, input_dim, z_dim):
        super().__init__()
        self.input_dim = input_dim
        self.z_dim = z_dim
        self.sigma_linear = nn.Linear(input_dim, z_dim)
        self.mu_linear = nn.Linear(input_dim, z_dim)
        self.return_means = False
        self.mu, self.sigma, self.z = None, None, None

    def forward(self, x, n=1, eps=None):
        self.mu = self.mu_linear(x)
        self.sigma = F.softplus(self.sigma_linear(x))
        self.z = self.nsample(n=n, eps=eps)
        return self.z

    def kl(self):
        return -0.5 * torch.sum(1 + 2 * self.sigma.log() - self.mu.pow(2) - self.sigma ** 2, -1)

    def log_posterior(self):
        return self._log_posterior(self.z)

    def _log_posterior(self, z):
        return Normal(self.mu, self.sigma).log_prob(z).sum(-1)

    def log_prior(self):
        return Normal(torch.zeros_like(self.mu), torch.ones_like(self.sigma)).log_prob(self.z).sum(-1)

    def nsample(self, n=1, eps=None):
        if self.return_means:
            return self.mu.expand(n, -1, -1)
        if eps is None:
            eps = torch.randn((n, *self.mu.shape), device=self.mu.device, dtype=self.mu.dtype)
        return self.mu + eps * self.sigma

    def deterministic(self):
        self.return_means = True


class Sreparameterize(nn.Module):
    """vMF latent (reparameterize.py:58-97) needs the third-party
    ``hyperspherical_vae_pytorch`` package, absent here and outside the SO(3) hot path."""

    def __init__(self, input_dim, z_dim):
        raise ImportError("Sreparameterize requires hyperspherical_vae_pytorch (out of scope, "
                          "see DESIGN.md)")


class N0reparameterize(nn.Module):
    """Zero-mean Gaussian in the algebra — reparameterize.py:100-145."""

    def __init__(self, input_dim, z_dim, fixed_sigma=None):
        super().__init__()
        self.input_dim = input_dim
        self.z_dim = z_dim
        self.sigma_linear = nn.Linear(input_dim, z_dim)
        self.return_means = False
        if fixed_sigma is not None:
            self.register_buffer('fixed_sigma', torch.tensor(fixed_sigma))
        else:
            self.fixed_sigma = None
        self.sigma = None
        self.z = None

    def forward(self, x, n=1, eps=None):
        if self.fixed_sigma is not None:
            self.sigma = x.new_full((x.shape[0], self.z_dim), float(self.fixed_sigma))
        else:
            self.sigma = _ops.unary(self.sigma_linear(x), _ops.SOFTPLUS)
        self.z = self.nsample(n=n, eps=eps)
        return self.z

    def kl(self):
        return -0.5 * torch.sum(1 + 2 * self.sigma.log() - self.sigma ** 2, -1)

    def log_posterior(self):
        return self._log_posterior(self.z)

    def _log_posterior(self, z):
        return Normal(torch.zeros_like(self.sigma), self.sigma).log_prob(z).sum(-1)

    def log_prior(self):
        return Normal(torch.zeros_like(self.sigma), torch.ones_like(self.sigma)).log_prob(self.z).sum(-1)

    def nsample(self, n=1, eps=None):
        if self.return_means:
            return torch.zeros_like(self.sigma).expand(n, -1, -1)
        if eps is None:
            eps = torch.randn((n, *self.sigma.shape), device=self.sigma.device,
                              dtype=self.sigma.dtype)
        if self.z_dim == 3:
            return _ops.n0_sample(self.sigma, eps)
        return eps * self.sigma


class AlgebraMean(nn.Module):
    """R^3 -> SO(3) through the exponential map — reparameterize.py:148-155."""

    def __init__(self, input_dims):
        super().__init__()
        self.map = nn.Linear(input_dims, 3)

    def forward(self, x):
        return rodrigues(self.map(x))


class QuaternionMean(nn.Module):
    """reparameterize.py:158-164."""

    def __init__(self, input_dims):
        super().__init__()
        self.map = nn.Linear(input_dims, 4)

    def forward(self, x):
        return quaternions_to_group_matrix(self.map(x))


class S2S1Mean(nn.Module):
    """reparameterize.py:167-181."""

    def __init__(self, input_dims):
        super().__init__()
        self.s2_map = nn.Linear(input_dims, 3)
        self.s1_map = nn.Linear(input_dims, 2)

    def forward(self, x):
        s2_el = self.s2_map(x)
        s2_el = s2_el / s2_el.norm(p=2, dim=-1, keepdim=True)
        s1_el = self.s1_map(x)
        s1_el = s1_el / s1_el.norm(p=2, dim=-1, keepdim=True)
        return s2s1rodrigues(s2_el, s1_el)


class S2S2Mean(nn.Module):
    """R^6 -> SO(3) by fp64 Gram–Schmidt — reparameterize.py:184-197."""

    def __init__(self, input_dims):
        super().__init__()
        self.map = nn.Linear(input_dims, 6)
        # Start with big outputs (reference :190-192)
        self.map.weight.data.uniform_(-10, 10)
        self.map.bias.data.uniform_(-10, 10)

    def forward(self, x):
        v = self.map(x).double().view(-1, 2, 3)
        return s2s2_gram_schmidt(v[:, 0], v[:, 1]).float()


class SO3reparameterize(nn.Module):
    """SO(3) latent z = μ·exp(v), v ~ N(0, σ) in the algebra — reparameterize.py:200-278."""

    def __init__(self, reparameterize, mean_module, k=10):
        super().__init__()
        self.mean_module = mean_module
        self.reparameterize = reparameterize
        self.input_dim = self.reparameterize.input_dim
        assert self.reparameterize.z_dim == 3
        self.k = k
        self.return_means = False
        self.mu_lie, self.v, self.z = None, None, None

    def forward(self, x, n=1, eps=None):
        self.mu_lie = self.mean_module(x)
        self.v = self.reparameterize(x, n, eps=eps) if eps is not None \
            else self.reparameterize(x, n)
        self.z = self.nsample(n=n)
        return self.z

    def kl(self):
        log_q_z_x = self.log_posterior()
        log_p_z = self.log_prior()
        kl = log_q_z_x - log_p_z
        return kl.mean(0)

    def log_posterior(self):
        """Wrapped density over 2k+1 sheets, fused into one HIP kernel (fwd + bwd)."""
        sigma = self.reparameterize.sigma
        v = self.v
        if v.dim() == 2:
            v = v.unsqueeze(0)
        return _ops.so3_log_posterior(v, sigma, self.k)

    def log_prior(self):
        # torch.tensor([-log 8pi^2], device=...) (reparameterize.py:265-267) is float64 (torch
        # infers it from the numpy scalar), so the KL and the IWAE weights are float64 there
        # too; a device fill of the same value keeps the dtype and needs no host-to-device
        # copy, so the step stays capturable in a hipGraph
        prior = self.z.new_full((1,), - np.log(8 * (np.pi ** 2)), dtype=torch.float64)
        return prior.expand_as(self.z[..., 0, 0])

    def nsample(self, n=1):
        if self.return_means:
            return self.mu_lie.expand(n, *[-1] * len(self.mu_lie.shape))
        return _ops.so3_sample(self.mu_lie, self.v)

    def deterministic(self):
        self.return_means = True
        self.reparameterize.deterministic()
