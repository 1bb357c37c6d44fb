"""Config-3 step diagnostics: per parameter group, the bf16 autocast step's clipped
gradient against the fp32 step's, for the default fused layers and with each library
layer family switched off (state_dict-identical models), plus the fp32 step's own
sensitivity to a 2^-9 relative perturbation of the input (how well conditioned each
group's gradient is).  MIOpen pinned deterministic.
  python tools/c3_step_diag.py [batch]"""
import copy
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "lie-vae_amd"), REPO]
from lie_vae.experiments import nets  # noqa: E402
from lie_vae.experiments.train_dp import DPTrainer  # noqa: E402
from lie_vae.experiments.vae import VAE  # noqa: E402

torch.backends.cudnn.deterministic = True
torch.backends.cudnn.benchmark = False
dev = torch.device("cuda:0")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
FLAGS = ("MFMA_DECONV", "FUSED_RELU", "FUSED_BN_ACT", "MFMA_CONV_DGRAD")
DEFAULT = {f: getattr(nets, f) for f in FLAGS}


def build(**flags):
    for f in FLAGS:
        setattr(nets, f, flags.get(f, DEFAULT[f]))
    torch.manual_seed(0)
    m = VAE(latent_mode="so3", decoder_mode="action", degrees=10, rep_copies=10, rgb=True,
            batch_norm=True, deconv_hidden=200, mean_mode="s2s2").to(dev)
    for f in FLAGS:
        setattr(nets, f, DEFAULT[f])
    return m.to(memory_format=torch.channels_last)


def groups(model):
    g = {}
    for name, _ in model.named_parameters():
        k = name.split(".")[0] if not name.startswith("decoder.") else (
            "item_rep" if name == "decoder.item_rep" else "deconv")
        if name.startswith("encoder."):
            k = "encoder." + name.split(".")[1]
        g.setdefault(k, []).append(name)
    return g


def step(model, x, eps, amp, clip=1e-5):
    tr = DPTrainer(model, lr=1e-3, clip_grads=clip, amp_dtype=amp)
    loss, _, _ = tr.step(x, eps)
    torch.cuda.synchronize()
    return float(loss), {k: p.grad.detach().double().clone() for k, p in model.named_parameters()}


base = build()
state = copy.deepcopy(base.state_dict())
G = groups(base)
gen = torch.Generator().manual_seed(21)
x = torch.rand(B, 3, 64, 64, generator=gen).to(dev)
eps = torch.randn(1, B, 3, generator=gen).to(dev)


def run(tag, amp, xx=x, clip=1e-5, **flags):
    m = build(**flags)
    m.load_state_dict(state)
    return step(m, xx, eps, amp, clip)


def err(a, b):
    out = {}
    for k, names in G.items():
        ga = torch.cat([a[n].flatten() for n in names])
        gb = torch.cat([b[n].flatten() for n in names])
        out[k] = round(float((ga - gb).norm() / gb.norm()), 5)
    return out


for clip in (1e-5, None):
    lf, gf = run("f32", None, clip=clip)
    rows = {"clip": clip, "f32_loss": lf,
            "f32_norms": {k: float(torch.cat([gf[n].flatten() for n in v]).norm()) for k, v in G.items()}}
    lp, gp = run("f32_pert", None, xx=x * (1 + 2.0 ** -9 * torch.randn_like(x)), clip=clip)
    rows["f32_input_perturbed"] = err(gp, gf)
    for tag, flags in (("bf16_default", {}), ("bf16_no_fused_bn", {"FUSED_BN_ACT": False}),
                       ("bf16_no_conv_dgrad", {"MFMA_CONV_DGRAD": False}),
                       ("bf16_no_library", {f: False for f in FLAGS})):
        lb, gb = run(tag, torch.bfloat16, clip=clip, **flags)
        rows[tag] = {"loss_rel": abs(lb - lf) / abs(lf), **err(gb, gf)}
    print(json.dumps(rows), flush=True)
