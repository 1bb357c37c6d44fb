#!/usr/bin/env python3
"""Conditioning of the config-3 step's gradient groups.

test_config3_bf16_step_matches_fp32_step holds each parameter group's bf16-step gradient
to max(0.06, 16·kappa), kappa = how far the fp32 step's own gradient moves under a 2^-9
relative perturbation of the input.  This tool shows where a large kappa comes from: it
repeats the fp32 / perturbed fp32 / bf16 comparison (clipped gradients, same seeds as the
test) with the per-sample loss of the k samples whose S2S2 Gram-Schmidt input pair is the
most nearly parallel masked out (k = 0, 1, 2, 4, 8, 16), and for the other mean modes.

  python tools/bf16_step_cond.py > gpurun_out/bf16_step_cond.json
"""
import copy
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "lie-vae_amd"), REPO]

from lie_vae.experiments.train_dp import DPTrainer  # noqa: E402
from lie_vae.experiments.vae import VAE  # noqa: E402


def groups_of(model):
    g = {"encoder": [], "rep_group": [], "item_rep": [], "deconv": []}
    for name, _ in model.named_parameters():
        if name.startswith("encoder."):
            g["encoder"].append(name)
        elif name.startswith("rep_group."):
            g["rep_group"].append(name)
        elif name == "decoder.item_rep":
            g["item_rep"].append(name)
        else:
            g["deconv"].append(name)
    return g


def clipped_grads(base, x, eps, amp, mask, clip=1e-5):
    m = copy.deepcopy(base)
    tr = DPTrainer(m, lr=1e-3, clip_grads=clip, amp_dtype=amp)
    gs = {}
    hook = None
    mm = m.reparameterize[0].mean_module
    if hasattr(mm, "map") and mm.map.out_features == 6:
        hook = mm.map.register_forward_hook(lambda mod, i, o: gs.__setitem__("v", o.detach().double()))
    tr.ar.zero_grad()
    ctx = torch.autocast("cuda", dtype=amp, cache_enabled=False) if amp else torch.autocast("cuda", enabled=False)
    with ctx:
        recon, kl, _ = m.elbo(x, 1, eps=eps)
    per = (recon.float() + kl.float()).reshape(-1)
    loss = (per * mask).sum() / mask.sum()
    loss.backward()
    tr.ar.finish()
    torch.nn.utils.clip_grad_norm_(m.parameters(), clip)
    torch.cuda.synchronize()
    if hook is not None:
        hook.remove()
    grads = {k: p.grad.detach().double().flatten().clone() for k, p in m.named_parameters()}
    return grads, gs.get("v"), float(loss)


def main():
    dev = torch.device("cuda", 0)
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = False
    out = {}
    for mean_mode in ("s2s2", "alg", "q"):
        torch.manual_seed(0)
        base = VAE(latent_mode="so3", decoder_mode="action", degrees=10, rep_copies=10, rgb=True,
                   batch_norm=True, deconv_hidden=200, mean_mode=mean_mode).to(dev)
        base = base.to(memory_format=torch.channels_last)
        groups = groups_of(base)
        g = torch.Generator().manual_seed(21)
        B = 512
        x = torch.rand(B, 3, 64, 64, generator=g).to(dev)
        eps = torch.randn(1, B, 3, generator=g).to(dev)
        xp = x * (1 + 2.0 ** -9 * torch.randn(x.shape, generator=g).to(dev))
        ones = torch.ones(B, device=dev)
        gf, v, _ = clipped_grads(base, x, eps, None, ones)
        order = None
        if v is not None:
            a, b = v[:, :3], v[:, 3:]
            sin = torch.linalg.cross(a, b, dim=-1).norm(dim=-1) / (a.norm(dim=-1) * b.norm(dim=-1))
            order = torch.argsort(sin)
            out.setdefault("s2s2_sin_smallest", sin[order[:16]].tolist())
        res = {}
        for k in ((0, 1, 2, 4, 8, 16) if order is not None else (0,)):
            mask = ones.clone()
            if k:
                mask[order[:k]] = 0
            f, _, lf = clipped_grads(base, x, eps, None, mask)
            p, _, _ = clipped_grads(base, xp, eps, None, mask)
            bb, _, lb = clipped_grads(base, x, eps, torch.bfloat16, mask)
            r = {"loss_rel": abs(lb - lf) / abs(lf)}
            for gname, names in groups.items():
                cf = torch.cat([f[n] for n in names])
                cp = torch.cat([p[n] for n in names])
                cb = torch.cat([bb[n] for n in names])
                r[gname] = {"kappa": float((cp - cf).norm() / cf.norm()),
                            "grad_bf16": float((cb - cf).norm() / cf.norm())}
            res[f"mask_{k}"] = r
            print(mean_mode, k, json.dumps(r), file=sys.stderr, flush=True)
        out[mean_mode] = res
        del base
        torch.cuda.empty_cache()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
