"""World-size-2 gloo tests (CPU) of the data-parallel training step (train_dp.py).

The kernels themselves need a GPU, so these tests drive the trainer's exchange logic
with a small torch-only stand-in model that has the same interface (``elbo``): the
bucketed async all-reduce must give every rank the gradient of the *global* batch mean,
clip by the global norm and keep the replicas bit-identical.
"""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn

from lie_vae.experiments import train_dp


class TinyVAE(nn.Module):
    """Stand-in with the VAE's elbo() contract: recon (B,) and kl (B,)."""

    def __init__(self):
        super().__init__()
        self.enc = nn.Sequential(nn.Linear(12, 16), nn.Tanh(), nn.Linear(16, 6))
        self.dec = nn.Linear(3, 12)
        self.unused = nn.Linear(2, 2)  # never gets a gradient: its bucket must still reduce

    def elbo(self, x, n=1, eps=None):
        h = self.enc(x)
        mu, logs = h[:, :3], h[:, 3:]
        z = mu + (eps if eps is not None else 0.0) * logs.exp()
        recon = (self.dec(z) - x).square().sum(-1)
        kl = 0.5 * (mu.square() + (2 * logs).exp() - 2 * logs - 1).sum(-1)
        return recon, kl, [kl]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, outdir, bucket_bytes, clip):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(100 + rank)  # different init per rank: broadcast must fix it
    model = TinyVAE()
    tr = train_dp.DPTrainer(model, lr=1e-2, clip_grads=clip, bucket_bytes=bucket_bytes)
    g = torch.Generator().manual_seed(7)
    for _ in range(3):
        xg = torch.randn(8, 12, generator=g)
        eg = torch.randn(8, 3, generator=g)
        tr.step(train_dp.shard(xg, rank, world), train_dp.shard(eg, rank, world))
    torch.save({k: v.clone() for k, v in model.state_dict().items()},
               os.path.join(outdir, f"rank{rank}.pt"))
    dist.destroy_process_group()


def _single(outdir, clip):
    torch.manual_seed(100)
    model = TinyVAE()
    opt = torch.optim.Adam(model.parameters(), lr=1e-2)
    g = torch.Generator().manual_seed(7)
    for _ in range(3):
        xg = torch.randn(8, 12, generator=g)
        eg = torch.randn(8, 3, generator=g)
        opt.zero_grad()
        recon, kl, _ = model.elbo(xg, eps=eg)
        (recon + kl).mean().backward()
        if clip:
            torch.nn.utils.clip_grad_norm_(model.parameters(), clip)
        opt.step()
    return model.state_dict()


@pytest.mark.parametrize("bucket_bytes,clip", [(1 << 20, None), (256, 1e-1)])
def test_dp_world2_matches_single_process(bucket_bytes, clip):
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(2, port, d, bucket_bytes, clip), nprocs=2, join=True)
        r0 = torch.load(os.path.join(d, "rank0.pt"), weights_only=True)
        r1 = torch.load(os.path.join(d, "rank1.pt"), weights_only=True)
        ref = _single(d, clip)
    for k in ref:
        assert torch.equal(r0[k], r1[k]), f"replicas diverged at {k}"
        torch.testing.assert_close(r0[k], ref[k], rtol=1e-5, atol=1e-6)


def test_bucket_plan_for_config3_model():
    """Flat fp32 gradient of the config-3 model (l=10, C=10, deconv_hidden=200) and its
    buckets: SURVEY.md §8(e) quotes 7,552,372 params = 30.2 MB."""
    import torch.nn as nn  # noqa: F401
    from lie_vae.experiments.vae import VAE
    m = VAE(latent_mode="so3", decoder_mode="action", degrees=10, rep_copies=10, rgb=True,
            batch_norm=True, deconv_hidden=200, mean_mode="s2s2")
    n = train_dp.param_count(m)
    assert n == 7552372 + 0 or abs(n - 7552372) < 2000, n
    sizes = train_dp.bucket_plan(m)
    assert sum(sizes) == 4 * n and len(sizes) >= 1
    assert train_dp.ring_bytes_per_rank(4 * n, 8) == pytest.approx(2 * 7 / 8 * 4 * n)
