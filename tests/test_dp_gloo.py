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
    """Stand-in with the VAE's contract: encoder, rep_group, forward, recon_loss, elbo()
    returning recon (B,) and kl (B,)."""

    def __init__(self):
        super().__init__()
        self.encoder = nn.Sequential(nn.Linear(12, 16), nn.Tanh(), nn.Linear(16, 6))
        self.rep_group = nn.Linear(6, 6)
        self.dec = nn.Linear(3, 12)
        self.unused = nn.Linear(2, 2)  # never gets a gradient: its bucket must still reduce

    def forward(self, x, n=1, eps=None):
        h = self.rep_group(self.encoder(x))
        mu, logs = h[:, :3], h[:, 3:]
        z = mu + (eps if eps is not None else 0.0) * logs.exp()
        self._kl = 0.5 * (mu.square() + (2 * logs).exp() - 2 * logs - 1).sum(-1)
        return self.dec(z)

    def recon_loss(self, x_recon, x):
        return (x_recon - x).square().sum(-1)

    def elbo(self, x, n=1, eps=None):
        x_recon = self.forward(x, n, eps)
        return self.recon_loss(x_recon, x), self._kl, [self._kl]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


TRAIN_KW = {
    "plain": {},
    "control": {"beta": None, "control": 0.5, "control_p": 2, "selective_clip": True},
    "control1": {"beta": None, "control": 0.3, "control_p": 1},
}


def _beta(kind):
    # a ramp that starts at 0 so that step 1 takes the recon-only branch
    # (unsupervised.py:80-83), then rises (LinearSchedule, experiments/utils.py:60-71)
    return train_dp.LinearSchedule(0.0, 2.0, 1, 3) if kind != "plain" else 1.0


def _worker(rank, world, port, outdir, bucket_bytes, clip, kind="plain"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(100 + rank)  # different init per rank: broadcast must fix it
    model = TinyVAE()
    kw = dict(TRAIN_KW[kind])
    kw["beta"] = _beta(kind)
    tr = train_dp.DPTrainer(model, lr=1e-2, clip_grads=clip, bucket_bytes=bucket_bytes, **kw)
    g = torch.Generator().manual_seed(7)
    for _ in range(3):
        xg = torch.randn(8, 12, generator=g)
        eg = torch.randn(8, 3, generator=g)
        tr.step(train_dp.shard(xg, rank, world), train_dp.shard(eg, rank, world))
    torch.save({k: v.clone() for k, v in model.state_dict().items()},
               os.path.join(outdir, f"rank{rank}.pt"))
    dist.destroy_process_group()


def _single(outdir, clip, kind="plain"):
    """The reference step, written out as unsupervised.py:69-117 does it."""
    torch.manual_seed(100)
    model = TinyVAE()
    opt = torch.optim.Adam(model.parameters(), lr=1e-2)
    kw = TRAIN_KW[kind]
    sched = _beta(kind)
    sched = sched if callable(sched) else (lambda it, b=sched: b)
    g = torch.Generator().manual_seed(7)
    for it in range(3):
        xg = torch.randn(8, 12, generator=g)
        eg = torch.randn(8, 3, generator=g)
        beta = sched(it + 1)
        opt.zero_grad()
        if beta == 0:
            recon = model.recon_loss(model.forward(xg, 1, eg), xg)
            kl = torch.zeros_like(recon)
        else:
            recon, kl, _ = model.elbo(xg, eps=eg)
        control = kw.get("control")
        if control is None:
            loss = (recon + beta * kl).mean()
        elif kw["control_p"] == 1:
            loss = (recon + control * torch.abs(beta - kl)).mean()
        else:
            loss = (recon + control * (beta - kl) ** 2).mean()
        loss.backward()
        if clip:
            params = (list(model.encoder.parameters()) + list(model.rep_group.parameters())
                      if kw.get("selective_clip") else model.parameters())
            torch.nn.utils.clip_grad_norm_(params, clip)
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


@pytest.mark.parametrize("kind,clip", [("control", 1e-1), ("control1", None)])
def test_dp_world2_reference_step_semantics(kind, clip):
    """beta schedule (incl. the beta == 0 recon-only step), KL control p in {1, 2} and
    selective clipping over encoder + rep_group, at world 2 against the single-process
    reference step."""
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(2, port, d, 256, clip, kind), nprocs=2, join=True)
        r0 = torch.load(os.path.join(d, "rank0.pt"), weights_only=True)
        r1 = torch.load(os.path.join(d, "rank1.pt"), weights_only=True)
        ref = _single(d, clip, kind)
    for k in ref:
        assert torch.equal(r0[k], r1[k]), f"replicas diverged at {k}"
        torch.testing.assert_close(r0[k], ref[k], rtol=1e-5, atol=1e-6)


def test_linear_schedule_matches_reference_rule():
    """experiments/utils.py:88-105 test_linear_schedule, restated."""
    s = train_dp.LinearSchedule(4, 10, 1, 4)
    assert s(0) == 4 and s(1) == 4 and s(2) == 6 and s(4) == 10 and s(5) == 10
    s = train_dp.LinearSchedule(10, 4, 1, 4)
    assert s(0) == 10 and s(2) == 8 and s(5) == 4


def _capture_worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    tr = train_dp.DPTrainer(TinyVAE(), lr=1e-2, graph=True)
    try:
        tr.capture(torch.randn(4, 12))
        msg = "no error"
    except ValueError as e:
        msg = str(e)
    with open(os.path.join(outdir, f"cap{rank}.txt"), "w") as f:
        f.write(msg)
    dist.destroy_process_group()


def test_capture_refuses_uncapturable_collective():
    """A gloo all-reduce cannot be recorded in a hipGraph: capture() at world > 1 refuses
    any backend but nccl (RCCL) with a ValueError before touching the device."""
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_capture_worker, args=(2, port, d), nprocs=2, join=True)
        for r in range(2):
            with open(os.path.join(d, f"cap{r}.txt")) as f:
                assert "needs the nccl" in f.read()


def test_cached_cast_sink_once_per_parameter():
    """ADVICE r4 (nets._CachedCast): a parameter is counted by its bucket once per step,
    after every contribution is in the bucket.  Used once or twice through its cached bf16
    copy -- and beside a direct use -- the gradient lands in the bucket view and the
    post-accumulate hook (which autograd fires once, after all paths into the leaf) counts
    it once; a second count in one step raises instead of racing the bucket's
    all-reduce."""
    from lie_vae.experiments import nets
    p = nn.Parameter(torch.randn(5))
    ar = train_dp.BucketedAllReduce([p])
    counted = []
    ar._launch = lambda st: counted.append(torch.clone(p.grad))  # what the all-reduce would send
    pb = p.detach().to(torch.bfloat16)
    cases = [
        (lambda: (nets._CachedCast.apply(p, pb).float() * 2).sum(), 2.0),
        (lambda: (nets._CachedCast.apply(p, pb).float() * 2).sum()
         + (nets._CachedCast.apply(p, pb).float() * 3).sum(), 5.0),
        (lambda: (nets._CachedCast.apply(p, pb).float() * 2).sum() + (p * 4).sum(), 6.0),
    ]
    for make, want in cases:
        ar.zero_grad()
        counted.clear()
        make().backward()
        assert ar.state[0]["left"] == 0
        assert len(counted) == 1, "bucket launched more or less than once"
        assert torch.equal(counted[0], torch.full((5,), want)), (counted[0], want)
        with pytest.raises(RuntimeError, match="counted twice"):
            ar._on_grad(p)
