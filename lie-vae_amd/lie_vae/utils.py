"""Drop-in for ``lie_vae.utils`` (reference lie_vae/utils.py)."""
import torch


def logsumexp(inputs, dim=None, keepdim=False):
    """Max-shifted logsumexp — lie_vae/utils.py:4-26.

    Inside the SO(3) log-posterior the same reduction runs fused in the HIP kernel."""
    if dim is None:
        inputs = inputs.reshape(-1)
        dim = 0
    s, _ = torch.max(inputs, dim=dim, keepdim=True)
    outputs = s + (inputs - s).exp().sum(dim=dim, keepdim=True).log()
    if not keepdim:
        outputs = outputs.squeeze(dim)
    return outputs
