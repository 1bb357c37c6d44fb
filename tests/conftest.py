"""Shared test setup: path wiring, the ``gpu`` marker and fixture loading."""
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_ROOT = os.path.join(REPO, "lie-vae_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (PKG_ROOT, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    # MIOpen immediate mode off the find-db shipped with the package, as bench.py and
    # bench_train.py run it (before any convolution in this process); without it some NHWC
    # bf16 shapes take MIOpen's naive fallback kernels (~1.5 s per config-3 step)
    try:
        from lie_vae.experiments import nets
        nets.use_packaged_miopen_db()
    except ImportError:
        pass


def golden(name):
    with np.load(os.path.join(GOLDEN, name)) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def gpu_device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")
