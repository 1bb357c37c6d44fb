"""Toy spectrum dataset (reference lie_vae/experiments/datasets.py:129-162, ``ToyDataset``).

The one dataset of the reference that is *produced* by the hot path: Haar-random poses q,
one shared random spectrum scaled to Frobenius norm 10, and targets
x = block_wigner_matrix_multiply(quaternions_to_eazyz(q), spectrum, degrees).  Both maps
run in liblievae_hip.so, so ``generate`` needs a GPU device (the product path has no CPU
fallback).  The on-disk image datasets (spherecube / ShapeNet readers) are out of scope
(DESIGN.md §7): their files are absent and they never touch the SO(3) kernels.
"""
import torch
from torch.utils.data import TensorDataset

from ..lie_tools import block_wigner_matrix_multiply, quaternions_to_eazyz, random_quaternions


def toy_harmonics(degrees=6, rep_copies=10, device=None):
    """Spectrum ((degrees+1)^2, rep_copies) with norm 10, drawn from the CURRENT RNG
    stream of ``device`` (datasets.py:146-147); the caller seeds (datasets.py:144-145)."""
    h = torch.randn((degrees + 1) ** 2, rep_copies, device=device)
    return h / h.norm() * 10


class ToyDataset(TensorDataset):
    """Tensors (q (n,4), harmonics (n,M,C) stride-0 expand, x (n,M,C))."""
    num_workers = 0
    single_id = True
    rgb = False

    def __init__(self, tensors=None, device=None, path='data/toy.pt'):
        if tensors is None:
            # The reference pickles with torch.save; here only tensor payloads are read
            # back (weights_only=True executes nothing from the file).
            tensors = torch.load(path, weights_only=True)
        if device is not None:
            tensors = [t.to(device) for t in tensors]
        super().__init__(*tensors)

    @classmethod
    def generate(cls, n=1000, degrees=6, rep_copies=10, device=None, batch_size=64):
        """datasets.py:143-158: seed 0, spectrum first, then one Haar batch of poses per
        ``batch_size`` chunk, each pushed through the fused ZYZ + Wigner-D action."""
        # One seed, then spectrum and every pose batch from the same device stream, in the
        # reference's order (datasets.py:144-151): torch.manual_seed(0) seeds the CPU and
        # every CUDA generator, exactly like the reference's manual_seed + cuda.manual_seed.
        torch.manual_seed(0)
        harmonics = toy_harmonics(degrees, rep_copies, device)
        xs, qs = [], []
        for i in range(0, n, batch_size):
            batch_n = min(i + batch_size, n) - i
            q = random_quaternions(batch_n, device=device)
            x = block_wigner_matrix_multiply(
                quaternions_to_eazyz(q), harmonics.expand(batch_n, -1, -1), degrees)
            xs.append(x)
            qs.append(q)
        return cls(tensors=(torch.cat(qs, 0), harmonics.expand(n, -1, -1), torch.cat(xs, 0)),
                   device=device)

    def save(self, path='data/toy.pt'):
        q, h, x = self.tensors
        torch.save((q.cpu(), h.cpu().contiguous(), x.cpu()), path)
