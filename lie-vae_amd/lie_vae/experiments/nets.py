"""Encoder / decoder stacks used around the SO(3) latent — drop-in for
``lie_vae.experiments.nets`` (reference lie_vae/experiments/nets.py:7-90).

These dense convolutions are MFMA work and run through PyTorch-ROCm (MIOpen /
hipBLASLt); they are callers of the hot path, not part of it.
"""
from torch import nn


class View(nn.Module):
    def __init__(self, *shape):
        super().__init__()
        self.shape = shape

    def forward(self, x):
        return x.view(*self.shape)


class Flatten(nn.Module):
    def forward(self, x):
        return x.view(x.size(0), -1)


def _down_stack(in_dims, hidden, out_dims, batch_norm):
    """64x64 -> 4x4 by four stride-2 4x4 convs (widths h, 2h, 4h, 8h), then 4x4 -> 1x1."""
    layers, c = [], in_dims
    for i, width in enumerate([hidden, hidden * 2, hidden * 4, hidden * 8]):
        layers.append(nn.Conv2d(c, width, 4, 2, 1))
        if batch_norm:
            layers.append(nn.BatchNorm2d(width))
        layers.append(nn.LeakyReLU(0.2, inplace=True))
        c = width
    layers += [nn.Conv2d(c, out_dims, 4, 1, 0), Flatten()]
    return layers


class ConvNet(nn.Sequential):
    """nets.py:7-31 (no batch norm)."""

    def __init__(self, out_dims, hidden_dims=50, rgb=False):
        super().__init__(*_down_stack(3 if rgb else 1, hidden_dims, out_dims, False))


class ConvNetBN(nn.Sequential):
    """nets.py:33-57 (batch norm after every strided conv)."""

    def __init__(self, out_dims, hidden_dims=50, rgb=False):
        super().__init__(*_down_stack(3 if rgb else 1, hidden_dims, out_dims, True))


class DeconvNet(nn.Sequential):
    """1x1 -> 64x64 transposed-conv stack — nets.py:60-75."""

    def __init__(self, in_dims, hidden_dims, rgb=False):
        layers = [View(-1, in_dims, 1, 1), nn.ConvTranspose2d(in_dims, hidden_dims, 4, 1, 0), nn.ReLU()]
        for _ in range(3):
            layers += [nn.ConvTranspose2d(hidden_dims, hidden_dims, 4, 2, 1), nn.ReLU()]
        layers.append(nn.ConvTranspose2d(hidden_dims, 3 if rgb else 1, 4, 2, 1))
        super().__init__(*layers)


class MLP(nn.Sequential):
    """nets.py:78-90."""

    def __init__(self, input_dims, output_dims, hidden_dims, num_layers=1, activation=nn.ReLU):
        if num_layers == 0:
            super().__init__(nn.Linear(input_dims, output_dims))
            return
        layers = [nn.Linear(input_dims, hidden_dims), activation()]
        for _ in range(num_layers - 1):
            layers += [nn.Linear(hidden_dims, hidden_dims), activation()]
        layers.append(nn.Linear(hidden_dims, output_dims))
        super().__init__(*layers)
