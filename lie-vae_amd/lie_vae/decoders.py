"""Decoders — drop-in for ``lie_vae.decoders`` (reference lie_vae/decoders.py)."""
import torch
from torch import nn as nn

from . import _ops
from .experiments.nets import MLP


class ActionNet(nn.Module):
    """Group-action decoder — decoders.py:9-61.

    ``item_rep`` ((degrees+1)^2 x rep_copies Fourier coefficients) is acted on by the
    block-diagonal real Wigner-D of the input ZYZ angles, flattened, optionally passed
    through an MLP, then through ``deconv``.  The action runs in one HIP kernel
    (forward) / one kernel + a deterministic reduction (backward); the stride-0
    ``item_rep.expand`` of the reference is passed once, not per sample.

    Extension: ``forward(angles, z_content=None)`` accepts and ignores a content
    vector, which is how the reference VAE calls it (vae.py:190; the reference's
    one-argument signature raises there — SURVEY.md Appendix B.2).
    """

    def __init__(self, degrees, deconv, rep_copies=10, with_mlp=False, item_rep=None,
                 transpose=False):
        super().__init__()
        self.degrees = degrees
        self.rep_copies = rep_copies
        self.matrix_dims = (degrees + 1) ** 2
        self.transpose = transpose
        if item_rep is None:
            self.item_rep = nn.Parameter(torch.randn((self.matrix_dims, rep_copies)))
        else:
            self.register_buffer('item_rep', item_rep)
        self.mlp = MLP(self.matrix_dims * rep_copies, self.matrix_dims * rep_copies, 50, 3) \
            if with_mlp else None
        self.deconv = deconv

    def harmonics(self, angles):
        """D(g)·item_rep flattened to (n, M*C) — decoders.py:53-56."""
        n, d = angles.shape
        assert d == 3, 'Input should be Euler angles.'
        out = _ops.group_action(angles, self.item_rep, self.degrees, transpose=self.transpose)
        return out.view(-1, self.matrix_dims * self.rep_copies)

    def harmonics_fused(self, mu, v):
        """The same harmonics for z = mu·exp(v) straight from (mu, v): exp, Euler
        extraction and the action in ONE launch (lv_fused_exp_action_fwd), instead of
        so3_sample -> group_matrix_to_eazyz -> group_action (reparameterize.py:269-273,
        vae.py:182, decoders.py:53-56).  mu (N,3,3) or None (identity), v (N,3)."""
        out = _ops.fused_exp_action(mu, v, self.item_rep, self.degrees, transpose=self.transpose)
        return out.view(-1, self.matrix_dims * self.rep_copies)

    def forward(self, angles, z_content=None):
        item = self.harmonics(angles)
        if self.mlp:
            item = self.mlp(item)
        return self.deconv(item)

    def forward_fused(self, mu, v):
        """forward() for z = mu·exp(v) given as (mu, v); see harmonics_fused."""
        item = self.harmonics_fused(mu, v)
        if self.mlp:
            item = self.mlp(item)
        return self.deconv(item)


class MLPNet(nn.Module):
    """Baseline decoder (group element -> MLP -> deconv) — decoders.py:64-87."""

    def __init__(self, degrees, deconv, in_dims=9, rep_copies=10, layers=3, hidden_dims=50,
                 activation=nn.ReLU):
        super().__init__()
        matrix_dims = (degrees + 1) ** 2
        self.mlp = MLP(in_dims, matrix_dims * rep_copies, hidden_dims, layers, activation)
        self.deconv = deconv

    def forward(self, x, content_data=None):
        n = x.size(0)
        return self.deconv(self.mlp(x.view(n, -1)))
