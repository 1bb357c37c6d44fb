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

import numpy as np
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
                # the gradient view keeps its parameter's strides (a channels-last model's
                # 4-D weights): same layout as the parameter and its Adam state, which
                # torch's foreach / fused optimizer kernels require (else per-tensor loops)
                flat = buf[off:off + p.numel()]
                dense = p.is_contiguous() or (p.dim() == 4 and p.is_contiguous(memory_format=torch.channels_last))
                p.grad = flat.as_strided(p.shape, p.stride()) if dense else flat.view_as(p)
                self.owner[p] = bi
                off += p.numel()
            self.state.append({"buf": buf, "left": len(plist), "handle": None})
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in self.params]
        for p in self.params:  # .grad is a bucket view: nets._CachedCast may add into it
            p._lv_grad_sink = self._on_grad
        self._seen = set()

    def _on_grad(self, p):
        # once per parameter per step: a second call means a gradient arrived after its
        # bucket may already be in flight (silently lost from the all-reduce), so refuse it
        if p in self._seen:
            raise RuntimeError(
                "BucketedAllReduce: a parameter was counted twice in one step (a second "
                "backward without zero_grad?); its bucket's all-reduce may already be in "
                "flight.")
        self._seen.add(p)
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
        self._seen = set()

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


class ConstantSchedule:
    """beta(it) = value (experiments/utils.py ConstantSchedule)."""

    def __init__(self, value):
        self.value = value

    def __call__(self, it):
        return self.value


class LinearSchedule:
    """Linear ramp from (start_x, start_y) to (end_x, end_y), clipped to the y range
    (experiments/utils.py:60-71, same arithmetic: np.clip of the line)."""

    def __init__(self, start_y, end_y, start_x, end_x):
        self.min_y = min(start_y, end_y)
        self.max_y = max(start_y, end_y)
        self.start_x = start_x
        self.start_y = start_y
        self.coef = (end_y - start_y) / (end_x - start_x)

    def __call__(self, x):
        return float(np.clip((x - self.start_x) * self.coef + self.start_y,
                             self.min_y, self.max_y))


class DPTrainer:
    """Sharded-batch training step with the reference's loss, clip and optimizer.

    The step follows ``UnsupervisedExperiment.train`` (unsupervised.py:69-117):
      * beta = beta_schedule(global_it), global_it counted from 1 (unsupervised.py:77-78);
        a float is a constant schedule;
      * beta == 0: reconstruction only, kl = 0 (unsupervised.py:80-83);
      * control (KL-controlled VAE, unsupervised.py:87-95):
        p = 1: (recon + control·|beta − kl|).mean(); p = 2: (recon + control·(beta − kl)²).mean();
      * clip_grad_norm_ over all parameters, or over encoder + rep_group only with
        ``selective_clip`` (unsupervised.py:110-115) -- here by the GLOBAL norm, since the
        gradients are already all-reduced;
      * Adam step.
    The per-step NaN-KL check (unsupervised.py:97-98) forces a host sync; it is off by
    default and enabled with ``nan_check=True``.

    ``amp_dtype=torch.bfloat16`` runs the forward under autocast: the conv encoder,
    deconv decoder and linear layers compute on the bf16 MFMA path (fp32 accumulate, fp32
    master weights and Adam state), while the SO(3) kernels keep computing in fp32 (their
    autograd ops cast their inputs) and S2S2 in fp64.  Off by default: the reference
    trains in fp32.

    ``graph=True`` builds Adam with device-side step state (``capturable``) so that
    :meth:`capture` can record the whole step -- forward, backward, the bucketed
    all-reduce, clip and Adam -- as one hipGraph and replay it without host launches.

    ``sync_bn=True`` converts the encoder's BatchNorm layers to ``SyncBatchNorm``: batch
    statistics over the global batch (one all-gather of per-rank moments per layer), so
    the DP step equals the single-device step on the concatenated batch, as the
    reference's one-device training computes it.  Off by default: per-rank statistics
    need no forward collective.
    """

    def __init__(self, model, lr=1e-3, weight_decay=0.0, clip_grads=1e-5, beta=1.0,
                 elbo_samples=1, bucket_bytes=32 << 20, group=None, broadcast=True,
                 control=None, control_p=1, selective_clip=False, nan_check=False,
                 amp_dtype=None, graph=False, sync_bn=False, fused_adam=None):
        if sync_bn and dist.is_initialized() and dist.get_world_size(group) > 1:
            from .nets import to_sync_batchnorm
            model = to_sync_batchnorm(model, process_group=group)
        self.model = model
        self.amp_dtype = amp_dtype
        self.clip = clip_grads
        self.beta_schedule = beta if callable(beta) else ConstantSchedule(beta)
        self.n = elbo_samples
        if control is not None and control_p not in (1, 2):
            raise RuntimeError("Wrong control p")
        self.control, self.control_p = control, control_p
        self.selective_clip = selective_clip
        self.nan_check = nan_check
        self.it = 0
        if dist.is_initialized() and broadcast:
            for t in list(model.parameters()) + list(model.buffers()):
                dist.broadcast(t.data, src=0, group=group)
        self.ar = BucketedAllReduce(model.parameters(), bucket_bytes=bucket_bytes, group=group)
        # fused Adam (one kernel per dtype / device / layout group instead of the foreach
        # kernels' chain) for device parameters; fused_adam=False keeps torch's default
        # (foreach; an explicit fused=False would select the per-tensor loop)
        if fused_adam is None:
            fused_adam = all(p.is_cuda for p in model.parameters())
        self.opt = torch.optim.Adam(model.parameters(), lr=lr, weight_decay=weight_decay,
                                    capturable=graph, fused=True if fused_adam else None)
        self._graph = None
        # bf16 autocast: the conv parameters' bf16 copies, refreshed by one multi-tensor
        # copy after each optimizer step instead of one cast kernel per tensor per forward
        self.bf16_params = None
        if amp_dtype == torch.bfloat16 and all(p.is_cuda for p in model.parameters()):
            from .nets import Bf16ParamCache
            self.bf16_params = Bf16ParamCache(model)

    def loss(self, x, eps=None, beta=1.0):
        if self.amp_dtype is not None:
            # no autocast weight cache: the step may be captured into a graph
            with torch.autocast(device_type=x.device.type, dtype=self.amp_dtype,
                                cache_enabled=False):
                out = self._loss(x, eps, beta)
            # autocast may leave bf16 reductions; the fp32/fp64 terms keep their dtype
            return tuple(t.float() if t.dtype in (torch.bfloat16, torch.float16) else t
                         for t in out)
        return self._loss(x, eps, beta)

    def _loss(self, x, eps=None, beta=1.0):
        if beta == 0:
            x_recon = self.model.forward(x, self.n, eps=eps)
            recon = self.model.recon_loss(x_recon, x)
            kl = torch.zeros_like(recon)
        else:
            recon, kl, _ = self.model.elbo(x, n=self.n, eps=eps)
        if self.control is None:
            loss = (recon + beta * kl).mean()
        elif self.control_p == 1:
            loss = (recon + self.control * torch.abs(beta - kl)).mean()
        else:
            loss = (recon + self.control * (beta - kl) ** 2).mean()
        return loss, recon, kl

    def clip_params(self):
        if self.selective_clip:
            return list(self.model.encoder.parameters()) + \
                list(self.model.rep_group.parameters())
        return list(self.model.parameters())

    def step(self, x, eps=None):
        self.it += 1
        return self._step_body(x, eps, self.beta_schedule(self.it))

    def _step_body(self, x, eps, beta):
        self.ar.zero_grad()
        loss, recon, kl = self.loss(x, eps, beta)
        if self.nan_check and torch.isnan(kl).sum():
            raise RuntimeError("NaN KL")
        loss.backward()
        self.ar.finish()
        if self.clip:
            torch.nn.utils.clip_grad_norm_(self.clip_params(), self.clip)
        self.opt.step()
        if self.bf16_params is not None:
            self.bf16_params.refresh()
        return loss.detach(), recon.detach(), kl.detach()

    # ------------------------------------------------------------ graph capture
    def _state_tensors(self):
        ts = list(self.model.parameters()) + list(self.model.buffers())
        for p in self.model.parameters():
            ts += [t for t in self.opt.state.get(p, {}).values() if torch.is_tensor(t)]
        return ts

    # the per-forward samples the latent modules and the VAE keep on ``self``
    # (reparameterize.py:41,94-95,192; vae.py:103)
    _SAMPLE_FIELDS = ("z", "v", "mu_lie", "sigma", "mu")

    def _drop_autograd_refs(self):
        """The model keeps its last sample (VAE.z, the latent modules' z / v / mu_lie /
        sigma) with the autograd graph attached; that graph holds the parameters'
        AccumulateGrad nodes, which would then keep the eager stream and break capture on
        the side stream.  Only those known sample fields are detached; nothing else on the
        modules is touched."""
        def strip(v):
            if torch.is_tensor(v):
                return v.detach() if v.grad_fn is not None else v
            if isinstance(v, tuple) and hasattr(v, "_fields"):  # namedtuple
                return type(v)(*(strip(u) for u in v))
            if isinstance(v, (list, tuple)):
                return type(v)(strip(u) for u in v)
            return v
        for m in self.model.modules():
            for k in self._SAMPLE_FIELDS:
                if k in vars(m) and not isinstance(vars(m)[k], torch.nn.Module):
                    setattr(m, k, strip(vars(m)[k]))

    def capture(self, x, eps=None, warmup=3):
        """Record one training step as a hipGraph; returns ``replay(x=None, eps=None)``
        which copies new inputs into the graph's static buffers, replays the step and
        returns its (loss, recon, kl) tensors (overwritten by the next replay).

        The warm-up steps that capture needs (allocator pools, MIOpen solutions, lazy
        Adam state) run on a side stream and are then undone: parameters, buffers and
        optimizer state are restored in place, so the first replay is the step eager
        ``step`` would have taken from the same state.  Needs ``graph=True``, a constant
        non-zero beta and ``nan_check=False`` (the graph has no host branch)."""
        if not self.opt.defaults.get("capturable"):
            raise ValueError("capture() needs DPTrainer(graph=True) (capturable Adam)")
        if not isinstance(self.beta_schedule, ConstantSchedule) or self.beta_schedule.value == 0:
            raise ValueError("capture() needs a constant, non-zero beta")
        if self.nan_check:
            raise ValueError("capture() cannot run the per-step NaN check")
        if self.ar.world > 1 and dist.get_backend(self.ar.group) != "nccl":
            raise ValueError("capture() with world > 1 needs the nccl (RCCL) backend: a "
                             f"{dist.get_backend(self.ar.group)} all-reduce cannot be captured "
                             "in a hipGraph")
        beta = self.beta_schedule.value
        dev = x.device
        self._drop_autograd_refs()
        gx = x.detach().clone()
        geps = None if eps is None else eps.detach().clone()
        had_state = {p for p in self.model.parameters() if self.opt.state.get(p)}
        snap = [(t, t.detach().clone()) for t in self._state_tensors()]
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(warmup):
                self._step_body(gx, geps, beta)
        torch.cuda.current_stream(dev).wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            out = self._step_body(gx, geps, beta)
        torch.cuda.synchronize(dev)
        # undo warm-up + capture: the tensors that existed before, then fresh Adam state
        with torch.no_grad():
            for t, v in snap:
                t.copy_(v)
            for p in self.model.parameters():
                if p not in had_state:
                    for t in self.opt.state.get(p, {}).values():
                        if torch.is_tensor(t):
                            t.zero_()
        if self.bf16_params is not None:  # the graph's forward reads the copies: re-derive
            self.bf16_params.refresh()
        self._graph = graph

        def replay(x_new=None, eps_new=None):
            if x_new is not None:
                gx.copy_(x_new)
            if eps_new is not None:
                if geps is None:
                    raise ValueError("this graph was captured without eps (the model draws "
                                     "its own noise); capture with eps to inject it")
                geps.copy_(eps_new)
            self.it += 1
            graph.replay()
            return out
        return replay


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


__all__ = ["BucketedAllReduce", "DPTrainer", "ConstantSchedule", "LinearSchedule", "shard", "param_count", "bucket_plan",
           "ring_bytes_per_rank", "math"]
