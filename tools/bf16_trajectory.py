"""bf16 vs fp32 training trajectories of the config-3 VAE (tools only; the test is
tests/test_gpu_configs.py::test_config3_bf16_trajectory_matches_fp32).

K DPTrainer steps (reference step: unsupervised.py:108-117) from one init on the same
seeded batches, in fp32, fp32 with the input perturbed by 2^-9 (the fp32 step's own noise
floor) and bf16 autocast; per step the loss, at the end the per-group accumulated
parameter change and its cosine with the fp32 run's.  Writes gpurun_out/bf16_traj_<mode>.json.
  python tools/bf16_trajectory.py [steps] [mean_mode]
"""
import copy
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "lie-vae_amd"))
from lie_vae.experiments.train_dp import DPTrainer  # noqa: E402
from lie_vae.experiments.vae import VAE  # noqa: E402


def groups_of(model):
    g = {"encoder": [], "rep_group": [], "item_rep": [], "deconv": []}
    for name, _ in model.named_parameters():
        key = ("encoder" if name.startswith("encoder.") else "rep_group" if name.startswith("rep_group.")
               else "item_rep" if name == "decoder.item_rep" else "deconv")
        g[key].append(name)
    return g


def run(steps=50, mean_mode="s2s2", B=512, L=10, seed=0, dev="cuda:0", heads=(2,)):
    from lie_vae.experiments import vae as vae_mod
    from lie_vae.experiments import nets
    nets.use_packaged_miopen_db()
    torch.backends.cudnn.deterministic = os.environ.get("TRAJ_DET", "0") == "1"
    torch.backends.cudnn.benchmark = False
    import time
    t0 = time.time()
    torch.manual_seed(seed)
    base = VAE(latent_mode="so3", decoder_mode="action", degrees=L, rep_copies=10, rgb=True,
               batch_norm=True, deconv_hidden=200, mean_mode=mean_mode).to(dev)
    base = base.to(memory_format=torch.channels_last)
    groups = groups_of(base)
    p0 = {k: p.detach().clone() for k, p in base.named_parameters()}
    gen = torch.Generator(device=dev).manual_seed(seed + 1)
    xs = [torch.rand(B, 3, 64, 64, device=dev, generator=gen) for _ in range(steps)]
    es = [torch.randn(1, B, 3, device=dev, generator=gen) for _ in range(steps)]
    noise = [1 + 2.0 ** -9 * torch.randn(B, 3, 64, 64, device=dev, generator=gen) for _ in range(steps)]
    out = {}
    runs = [("f32", None, False, 0), ("f32_pert", None, True, 0)]
    runs += [("bf16" if h == heads[0] else f"bf16_heads{h}", torch.bfloat16, False, h) for h in heads]
    for tag, amp, pert, hd in runs:
        vae_mod.AMP_FP32_HEADS = hd
        m = copy.deepcopy(base)
        tr = DPTrainer(m, lr=1e-3, clip_grads=1e-5, amp_dtype=amp)
        losses = []
        for k in range(steps):
            loss, _, _ = tr.step(xs[k] * noise[k] if pert else xs[k], es[k])
            losses.append(loss.detach())
            if k % 5 == 0:
                print(tag, "step", k, float(loss), f"{time.time() - t0:.1f} s", flush=True)
        torch.cuda.synchronize()
        named = dict(m.named_parameters())
        out[tag] = {"loss": [float(x) for x in losses],
                    "delta": {g: torch.cat([(named[n].detach() - p0[n]).flatten() for n in names]).double()
                              for g, names in groups.items()}}
        del m, tr
    rep = {"steps": steps, "mean_mode": mean_mode, "batch": B}
    f = out["f32"]
    for tag in [t for t in out if t != "f32"]:
        o = out[tag]
        rel = [abs(a - b) / abs(b) for a, b in zip(o["loss"], f["loss"])]
        rep[tag] = {"loss_rel_max": max(rel), "loss_rel_last": rel[-1],
                    "loss_mean_rel": abs(sum(o["loss"]) - sum(f["loss"])) / abs(sum(f["loss"]))}
        for g in groups:
            a, b = o["delta"][g], f["delta"][g]
            rep[tag][g] = {"cos": float(a @ b / (a.norm() * b.norm())),
                           "rel": float((a - b).norm() / b.norm())}
    rep["loss_f32"] = f["loss"]
    rep["loss_bf16"] = out["bf16"]["loss"]
    return rep


if __name__ == "__main__":
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    mode = sys.argv[2] if len(sys.argv) > 2 else "s2s2"
    heads = tuple(int(h) for h in sys.argv[3].split(",")) if len(sys.argv) > 3 else (2,)
    rep = run(steps, mode, heads=heads)
    os.makedirs("gpurun_out", exist_ok=True)
    with open(f"gpurun_out/bf16_traj_{mode}.json", "w") as fh:
        json.dump(rep, fh, indent=1)
    for tag in [t for t in rep if t.startswith(("f32_pert", "bf16"))]:
        print(tag, json.dumps({k: v for k, v in rep[tag].items()}))
