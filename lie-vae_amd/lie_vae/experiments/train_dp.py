"""Data-parallel training step for the SO(3) VAE: one process per GPU, batch sharded.

The reference trains on one device (lie_vae/experiments/main.py:17) with the step of
unsupervised.py:69-117:
  loss = (recon + beta * kl).mean(); backward; clip_grad_norm_(params, clip); Adam.step.

Here every rank computes that loss on its own shard.  The one exchange step is a
bucketed all-reduce of the gradients (RCCL over xGMI when the process group is
``nccl``, gloo on CPU for tests).  Gradients live in flat per-bucket buffers: each
parameter's ``.grad`` is a view into one, so backward accumulates straight into the
buffer and a bucket's all-reduce is launched (async) from the post-accumulate hook of
its last parameter, overlapping the rest of backward.  Buckets follow reverse parameter
order (roughly the order backward produces them) and are sized for xGMI's ~150 GB/s
per-link rings (default 32 MiB: two buckets for the l=10 / deconv_hidden=200 model's
30 MB of fp32 gradients).  After the wait the buffers hold the sum; dividing by the
world size gives the gradient of the global-batch mean, so clipping by the *global*
norm and the Adam step are identical on every rank (replicas stay in lock-step).

No host synchronisation inside the step: loss terms stay on the device.
"""
import math

import torch
import torch.distributed as dist


class BucketedAllReduce:
    def __init__(self, params, bucket_bytes=32 << 20, group=None):
        self.params = [p for p in params if p.requires_grad]
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.buckets = []  # each: dict(params, buf, pending, handle)
        cur, cur_bytes = [], 0
        for p in reversed(self.params):
            nbytes = p.numel() * p.element_size()
            if cur and cur_bytes + nbytes > bucket_bytes:
                self.buckets.append(cur)
                cur, cur_bytes = [], 0
            cur.append(p)
            cur_bytes += nbytes
        if cur:
            self.buckets.append(cur)
        self.state = []
        self.owner = {}
        for bi, plist in enumerate(self.buckets):
            dtype = plist[0].dtype
            assert all(p.dtype == dtype and p.device == plist[0].device for p in plist)
            buf = torch.zeros(sum(p.numel() for p in plist), dtype=dtype, device=plist[0].device)
            off = 0
            for p in plist:
                p.grad = buf[off:off + p.numel()].view_as(p)
                self.owner[p] = bi
                off += p.numel()
            self.state.append({"buf": buf, "left": len(plist), "handle": None})
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in self.params]

    def _on_grad(self, p):
        st = self.state[self.owner[p]]
        st["left"] -= 1
        if st["left"] == 0:
            self._launch(st)

    def _launch(self, st):
        if self.world > 1 and st["handle"] is None:
            st["handle"] = dist.all_reduce(st["buf"], op=dist.ReduceOp.SUM, group=self.group,
                                           async_op=True)

    def zero_grad(self):
        for plist, st in zip(self.buckets, self.state):
            st["buf"].zero_()
            st["left"] = len(plist)
            st["handle"] = None

    def finish(self):
        """Wait for every bucket (launching any whose parameters got no gradient) and
        turn the sums into means."""
        for st in self.state:
            if st["handle"] is None:
                self._launch(st)
        for st in self.state:
            if st["handle"] is not None:
                st["handle"].wait()
            if self.world > 1:
                st["buf"].div_(self.world)

    def grad_norm(self):
        return torch.sqrt(sum(st["buf"].double().square().sum() for st in self.state))


class DPTrainer:
    """Sharded-batch training step with the reference's loss, clip and optimizer."""

    def __init__(self, model, lr=1e-3, weight_decay=0.0, clip_grads=1e-5, beta=1.0,
                 elbo_samples=1, bucket_bytes=32 << 20, group=None, broadcast=True):
        self.model = model
        self.clip = clip_grads
        self.beta = beta
        self.n = elbo_samples
        if dist.is_initialized() and broadcast:
            for t in list(model.parameters()) + list(model.buffers()):
                dist.broadcast(t.data, src=0, group=group)
        self.ar = BucketedAllReduce(model.parameters(), bucket_bytes=bucket_bytes, group=group)
        self.opt = torch.optim.Adam(model.parameters(), lr=lr, weight_decay=weight_decay)

    def loss(self, x, eps=None):
        recon, kl, _ = self.model.elbo(x, n=self.n, eps=eps)
        return (recon + self.beta * kl).mean(), recon, kl

    def step(self, x, eps=None):
        self.ar.zero_grad()
        loss, recon, kl = self.loss(x, eps)
        loss.backward()
        self.ar.finish()
        if self.clip:
            torch.nn.utils.clip_grad_norm_(self.model.parameters(), self.clip)
        self.opt.step()
        return loss.detach(), recon.detach(), kl.detach()


def shard(batch, rank, world):
    """Contiguous shard of a global batch for this rank (equal shards)."""
    n = batch.shape[0]
    assert n % world == 0, f"global batch {n} not divisible by world {world}"
    k = n // world
    return batch[rank * k:(rank + 1) * k]


def param_count(model):
    return sum(p.numel() for p in model.parameters())


def bucket_plan(model, bucket_bytes=32 << 20):
    """Bucket sizes (bytes) the trainer would use — for DESIGN.md / sizing checks."""
    sizes, cur = [], 0
    for p in reversed([p for p in model.parameters() if p.requires_grad]):
        b = p.numel() * p.element_size()
        if cur and cur + b > bucket_bytes:
            sizes.append(cur)
            cur = 0
        cur += b
    if cur:
        sizes.append(cur)
    return sizes


def ring_bytes_per_rank(total_bytes, world):
    return 2 * (world - 1) / world * total_bytes if world > 1 else 0.0


__all__ = ["BucketedAllReduce", "DPTrainer", "shard", "param_count", "bucket_plan",
           "ring_bytes_per_rank", "math"]
