"""GPU parity of BASELINE configurations 3 and 5 and of the remaining callers of the
boundary (latent mode ``normal``, the MLP decoders, ToyDataset's RNG stream, the fused
VAE decode), against the CPU oracle (oracle/lie_ref.py) on identical inputs.

Config 5 (l = 20, B = 8192, bf16 out, fp32 recursion): the timed kernel of that bench,
``lv_fused_exp_action_fwd`` with a bf16 output, checked on every row against the fp32
oracle at bf16 rounding tolerance, bitwise against its own fp32 output rounded to bf16,
and through norm preservation and D^T D F = F at full size.

Config 3 (conv VAE, B = 512): the SO(3) part (mean map -> sigma -> v -> z -> Euler ->
action) at 1e-5 against the oracle fed the GPU encoder's own features, so MIOpen's conv
numerics (Winograd etc.) do not pollute the hot-path parity; the convs themselves are
checked against CPU torch at a conv tolerance.  One DPTrainer step at world 1 must be
finite and repeatable.
"""
import copy
import json
import math
import os

import numpy as np
import pytest
import torch

from conftest import REPO
from test_gpu_parity import assert_normwise, assert_parity_fp64, host

pytestmark = pytest.mark.gpu

BF16_TOL = 2.0 ** -9 + 1e-5  # bf16 round-to-nearest (8 significant bits) + fp32 noise


# --------------------------------------------------------------------- config 5
@pytest.mark.parametrize("n", [8192, 1001])
def test_config5_fused_bf16_l20(gpu_device, n):
    import lie_vae._ops as ops
    import lie_vae.lie_tools as lt
    from oracle import lie_ref
    gen = torch.Generator().manual_seed(500 + n)
    L, C = 20, 10
    v = torch.randn(n, 3, generator=gen)
    F = torch.randn((L + 1) ** 2, C, generator=gen)
    vd, Fd = v.to(gpu_device), F.to(gpu_device)
    out = ops.fused_exp_action(None, vd, Fd, L, out_dtype=torch.bfloat16)
    out32 = ops.fused_exp_action(None, vd, Fd, L)
    assert out.dtype == torch.bfloat16 and out.shape == (n, (L + 1) ** 2, C)
    # the bf16 kernel is the fp32 chain rounded once (RNE) at the store
    same = (out == out32.to(torch.bfloat16)).float().mean().item()
    assert same >= 1 - 1e-6, f"bf16 output differs from rounded fp32 on {1 - same:.2e}"
    # every row against the fp32 reference pipeline (chunked: the dense l = 20 chain)
    o = host(out.float())
    o32 = host(out32)
    for a in range(0, n, 2048):
        b = min(n, a + 2048)
        ref = lie_ref.block_wigner_apply(lie_ref.mat_to_eazyz(lie_ref.so3_exp(v[a:b])),
                                         F.expand(b - a, -1, -1), L).numpy()
        assert_normwise(o[a:b], ref, BF16_TOL, what=f"config5 bf16 rows {a}:{b}")
        if a == 0:
            ref64 = lie_ref.block_wigner_apply(
                lie_ref.mat_to_eazyz(lie_ref.so3_exp(v[a:b].double())),
                F.double().expand(b - a, -1, -1), L).numpy()
            assert_parity_fp64(o32[a:b], ref, ref64, what="config5 fp32 fused l=20")
    # size-independent properties: D orthogonal per degree block, D^T D F = F
    ob = out.float()
    for l in (0, 7, 20):
        r0, r1 = l * l, (l + 1) * (l + 1)
        torch.testing.assert_close(ob[:, r0:r1].norm(dim=1),
                                   F[r0:r1].norm(dim=0).to(gpu_device).expand(n, -1),
                                   rtol=4e-3, atol=1e-3)
    ang = lt.group_matrix_to_eazyz(lt.rodrigues(vd))
    back = ops.group_action(ang, ob, L, transpose=True)
    err = (back - Fd).flatten(1).norm(dim=1) / Fd.norm()
    assert err.max().item() <= 4e-3, err.max().item()


# --------------------------------------------------------------------- config 3
def _capture(module, store, key):
    return module.register_forward_hook(lambda m, i, o: store.__setitem__(key, (i[0], o)))


def test_config3_conv_vae_b512(gpu_device):
    from lie_vae.experiments.vae import VAE
    from oracle import lie_ref
    L, C, B = 10, 10, 512
    torch.manual_seed(0)
    cpu = VAE(latent_mode="so3", decoder_mode="action", degrees=L, rep_copies=C, rgb=True,
              batch_norm=True, deconv_hidden=200, mean_mode="s2s2")
    with torch.no_grad():  # non-trivial running statistics (eval mode uses them)
        for m in cpu.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.running_mean.uniform_(-0.1, 0.1)
                m.running_var.uniform_(0.5, 1.5)
    cpu.eval()
    g = torch.Generator().manual_seed(1)
    x = torch.rand(B, 3, 64, 64, generator=g)
    eps = torch.randn(1, B, 3, generator=g)
    gvae = copy.deepcopy(cpu).to(gpu_device).eval()
    cap = {}
    hooks = [_capture(gvae.encoder, cap, "enc"), _capture(gvae.decoder.deconv, cap, "dec")]
    with torch.no_grad():
        recon, kl, _ = gvae.elbo(x.to(gpu_device), 1, eps=eps.to(gpu_device))
    for h in hooks:
        h.remove()
    h_gpu = cap["enc"][1].cpu()
    harm_gpu = cap["dec"][0].cpu()
    xr_gpu = cap["dec"][1].cpu()
    # (1) the encoder convs vs CPU torch (conv tolerance), on a 64-sample slice
    with torch.no_grad():
        h_cpu = cpu.encoder(x[:64])
    assert_normwise(h_gpu[:64].numpy(), h_cpu.numpy(), 1e-4, what="encoder (MIOpen vs CPU)")
    # (2) the SO(3) hot path at 1e-5, oracle fed the GPU features
    rep = cpu.rep_group
    with torch.no_grad():
        def pipeline(h, e, dt):
            m6 = rep.mean_module.map.to(dt)(h.to(dt)).double().view(-1, 2, 3)
            mu = lie_ref.gram_schmidt_s2s2(m6[:, 0], m6[:, 1]).to(dt)
            sig = lie_ref.n0_sigma(rep.reparameterize.sigma_linear.to(dt)(h.to(dt)))
            vv = lie_ref.n0_sample(sig, e.to(dt))
            z = lie_ref.so3_sample(mu, vv)
            ang = lie_ref.mat_to_eazyz(z.reshape(-1, 3, 3))
            harm = lie_ref.action_decode(ang, cpu.decoder.item_rep.to(dt), L)
            lq = lie_ref.so3_log_posterior(vv, sig, 10)
            return harm, (lq + math.log(8 * math.pi ** 2)).mean(0)
        harm32, kl32 = pipeline(h_gpu, eps, torch.float32)
        harm64, _ = pipeline(h_gpu, eps, torch.float64)
        rep.float()
    assert_parity_fp64(harm_gpu.numpy(), harm32.numpy(), harm64.numpy(),
                       what="config3 SO(3) path (s2s2 mean, fused decode)")
    np.testing.assert_allclose(host(kl), kl32.numpy(), rtol=1e-5, atol=1e-4)
    # (3) the deconv vs CPU torch on the same harmonics, and the summed-squares recon
    with torch.no_grad():
        xr_cpu = cpu.decoder.deconv(harm_gpu[:64])
    assert_normwise(xr_gpu[:64].numpy().reshape(64, -1), xr_cpu.numpy().reshape(64, -1), 1e-4,
                    what="deconv (MIOpen vs CPU)")
    rec_ref = ((xr_gpu - x) ** 2).sum((-1, -2, -3))
    np.testing.assert_allclose(host(recon).reshape(-1), rec_ref.numpy(), rtol=1e-4)


def test_config3_dp_trainer_step_world1(gpu_device):
    """One data-parallel trainer step (world 1, reference loss, global-norm clip 1e-5,
    Adam) on the config-3 model: finite, and the same twice from the same state.  MIOpen
    is pinned to deterministic algorithms for the comparison (its default backward-weight
    convolutions may accumulate in any order); the SO(3) kernels are deterministic by
    construction."""
    from lie_vae.experiments.train_dp import DPTrainer
    from lie_vae.experiments.vae import VAE
    det, bench = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    try:
        _dp_trainer_step_world1(gpu_device)
    finally:
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = det, bench


def _dp_trainer_step_world1(gpu_device):
    from lie_vae.experiments.train_dp import DPTrainer
    from lie_vae.experiments.vae import VAE
    torch.manual_seed(0)
    base = VAE(latent_mode="so3", decoder_mode="action", degrees=10, rep_copies=10, rgb=True,
               batch_norm=True, deconv_hidden=200, mean_mode="s2s2").to(gpu_device)
    g = torch.Generator().manual_seed(2)
    x = torch.rand(512, 3, 64, 64, generator=g).to(gpu_device)
    eps = torch.randn(1, 512, 3, generator=g).to(gpu_device)
    results = []
    for _ in range(2):
        m = copy.deepcopy(base)
        tr = DPTrainer(m, lr=1e-3, clip_grads=1e-5)
        loss, recon, kl = tr.step(x, eps)
        loss2, _, _ = tr.step(x, eps)
        torch.cuda.synchronize()
        assert torch.isfinite(loss) and torch.isfinite(loss2)
        assert torch.isfinite(recon).all() and torch.isfinite(kl).all()
        p = torch.cat([q.detach().flatten() for q in m.parameters()])
        assert torch.isfinite(p).all()
        results.append((float(loss), float(loss2), p))
    assert results[0][0] == pytest.approx(results[1][0], rel=1e-5)
    assert results[0][1] == pytest.approx(results[1][1], rel=1e-4)
    torch.testing.assert_close(results[0][2], results[1][2], rtol=1e-4, atol=1e-6)


# ------------------------------------------------------ other latent modes / decoders (f4)
def test_normal_latent_mode_vs_oracle(gpu_device):
    """latent_mode='normal' + action decoder: Nreparameterize (reparameterize.py:16-55),
    vector_to_eazyz (lie_tools.py:92-97), ActionNet, injected eps."""
    from lie_vae.experiments.vae import VAE
    from oracle import lie_ref
    L, B, n = 6, 24, 3
    torch.manual_seed(5)
    cpu = VAE(latent_mode="normal", decoder_mode="action", degrees=L, encode_mode="toy",
              deconv_mode="toy", rep_copies=10)
    x = torch.randn(B, (L + 1) ** 2, 10)
    eps = torch.randn(n, B, 3)
    gv = copy.deepcopy(cpu).to(gpu_device)
    with torch.no_grad():
        recon, kl, _ = gv.elbo(x.to(gpu_device), n, eps=eps.to(gpu_device))
        xr = gv.forward(x.to(gpu_device), n, eps=eps.to(gpu_device))

        def pipeline(dt):
            c = copy.deepcopy(cpu).to(dt)
            h = c.encoder(x.to(dt))
            mu = c.rep_group.mu_linear(h)
            sig = torch.nn.functional.softplus(c.rep_group.sigma_linear(h))
            z = mu + eps.to(dt) * sig
            ang = lie_ref.squash_to_eazyz(z.reshape(-1, 3))
            xr_ref = lie_ref.action_decode(ang, c.decoder.item_rep, L)
            kl_ref = -0.5 * torch.sum(1 + 2 * sig.log() - mu.pow(2) - sig ** 2, -1)
            return xr_ref, kl_ref
        xr32, kl32 = pipeline(torch.float32)
        xr64, _ = pipeline(torch.float64)
    assert_parity_fp64(host(xr).reshape(n * B, -1), xr32.numpy(), xr64.numpy(),
                       what="normal mode x_recon")
    np.testing.assert_allclose(host(kl), kl32.numpy(), rtol=1e-5, atol=1e-5)
    rec_ref = ((xr32.reshape(n, B, -1) - x.reshape(1, B, -1)) ** 2).sum(-1)
    np.testing.assert_allclose(host(recon), rec_ref.numpy(), rtol=1e-4)


def test_mlp_decoders_vs_oracle(gpu_device):
    """MLPNet (decoders.py:64-87) and ActionNet(with_mlp=True) (decoders.py:39-41,58-59)."""
    from lie_vae.decoders import ActionNet, MLPNet
    from oracle import lie_ref
    L, N = 5, 40
    torch.manual_seed(8)
    an = ActionNet(L, torch.nn.Sequential(), rep_copies=4, with_mlp=True)
    mn = MLPNet(L, torch.nn.Sequential(), in_dims=9, rep_copies=4)
    ang = lie_ref.mat_to_eazyz(lie_ref.haar_matrices(N))
    zmat = lie_ref.haar_matrices(N)
    with torch.no_grad():
        ya = copy.deepcopy(an).to(gpu_device)(ang.to(gpu_device))
        ym = copy.deepcopy(mn).to(gpu_device)(zmat.to(gpu_device))
        ref_a = an.mlp(lie_ref.action_decode(ang, an.item_rep, L))
        ref_m = mn.mlp(zmat.reshape(N, -1))
    assert_normwise(host(ya), ref_a.numpy(), 1e-5, what="ActionNet(with_mlp)")
    assert_normwise(host(ym), ref_m.numpy(), 1e-5, what="MLPNet")


def test_toy_dataset_reference_rng_stream(gpu_device):
    """ToyDataset.generate draws the spectrum and every pose batch from ONE seeded device
    stream, in the reference's order (datasets.py:144-151): replay that order with plain
    torch on the same device and compare bit for bit."""
    from lie_vae.experiments.datasets import ToyDataset
    from lie_vae.lie_tools import random_quaternions
    n, deg, C, bs = 150, 6, 10, 64
    ds = ToyDataset.generate(n=n, degrees=deg, rep_copies=C, device=gpu_device, batch_size=bs)
    torch.manual_seed(0)
    torch.cuda.manual_seed(0)
    h = torch.randn((deg + 1) ** 2, C, device=gpu_device)
    h = h / h.norm() * 10
    qs = [random_quaternions(min(i + bs, n) - i, device=gpu_device) for i in range(0, n, bs)]
    assert torch.equal(ds.tensors[1][0], h)
    assert torch.equal(ds.tensors[0], torch.cat(qs, 0))


def test_vae_fused_decode_matches_modular(gpu_device):
    """VAE.decode's one-launch path (z = mu·exp(v) -> action) against the modular path
    (so3_sample -> group_matrix_to_eazyz -> ActionNet), outputs and every gradient."""
    from lie_vae.experiments.vae import VAE
    L, B, n = 8, 64, 2
    torch.manual_seed(4)
    a = VAE(latent_mode="so3", decoder_mode="action", degrees=L, encode_mode="toy",
            deconv_mode="toy", rep_copies=10, mean_mode="q").to(gpu_device)
    b = copy.deepcopy(a)
    b.fused_decode = False
    x = torch.randn(B, (L + 1) ** 2, 10, device=gpu_device)
    eps = torch.randn(n, B, 3, device=gpu_device)
    outs = []
    for m in (a, b):
        recon, kl, _ = m.elbo(x, n, eps=eps)
        (recon.sum() + kl.sum()).backward()
        outs.append((recon.detach(), {k: p.grad.clone() for k, p in m.named_parameters()}))
    torch.testing.assert_close(outs[0][0], outs[1][0], rtol=2e-5, atol=1e-4)
    for k in outs[0][1]:
        assert_normwise(host(outs[0][1][k]).reshape(1, -1), host(outs[1][1][k]).reshape(1, -1),
                        1e-4, what=f"grad {k}")


def test_dp_trainer_bf16_autocast_step(gpu_device):
    """DPTrainer(amp_dtype=bf16): the convs run under autocast while the SO(3) kernels
    stay fp32 (their ops cast); two steps are finite and move the loss like fp32 does
    to within bf16 noise."""
    from lie_vae.experiments.train_dp import DPTrainer
    from lie_vae.experiments.vae import VAE
    torch.manual_seed(0)
    base = VAE(latent_mode="so3", decoder_mode="action", degrees=10, rep_copies=10, rgb=True,
               batch_norm=True, deconv_hidden=200, mean_mode="s2s2").to(gpu_device)
    g = torch.Generator().manual_seed(3)
    x = torch.rand(64, 3, 64, 64, generator=g).to(gpu_device)
    eps = torch.randn(1, 64, 3, generator=g).to(gpu_device)
    out = {}
    for amp in (None, torch.bfloat16):
        m = copy.deepcopy(base)
        tr = DPTrainer(m, lr=1e-3, clip_grads=1e-5, amp_dtype=amp)
        l1, r1, k1 = tr.step(x, eps)
        l2, _, _ = tr.step(x, eps)
        torch.cuda.synchronize()
        assert l1.dtype in (torch.float32, torch.float64)
        assert torch.isfinite(l1) and torch.isfinite(l2)
        assert all(torch.isfinite(p).all() for p in m.parameters())
        out[amp] = (float(l1), float(l2))
    assert out[torch.bfloat16][0] == pytest.approx(out[None][0], rel=2e-2)


# Config-3 benchmarked step (bench_train.py --amp bf16 --channels-last) against the fp32 step.
# bf16 bound: one bf16 rounding has unit roundoff u = 2^-9.  Along the longest path of a
# conv/BN parameter's gradient the bf16 step rounds about k = 80 times (each of the 9
# conv / deconv layers rounds its input, weight and output forward, and its upstream
# gradient, input and weight gradient backward; the 4 BN+LeakyReLU layers their output and
# input gradient; the 2 mean / sigma linears likewise).  Independent roundings give a
# normwise relative error near sqrt(k)·u = 1.7e-2 for a well-conditioned gradient.  How
# well conditioned each group's gradient is, is measured in the test itself: the fp32 step
# on x·(1 + 2^-9·xi) (one rounding-sized relative perturbation of the input) moves the
# group's gradient by kappa (relative).  k independent rounding-sized perturbations move it
# by about sqrt(k)·kappa, so each group is held to
#     ||g_bf16 - g_f32|| / ||g_f32|| <= max(BF16_STEP_TOL, BF16_STEP_K · kappa),
# BF16_STEP_TOL = 0.06 (between sqrt(k)·u and the first-order worst case k·u = 0.16) and
# BF16_STEP_K = 16 (sqrt(80) = 9, with margin for the deeper roundings' own amplification).
BF16_STEP_TOL = 0.06
BF16_STEP_K = 16.0
BF16_KAPPA_MAX = 0.01
# Groups whose fp32 gradient is itself ill-conditioned at this initialisation (kappa >
# BF16_KAPPA_MAX: encoder 1.16, rep_group 0.053, item_rep 0.075 -- DESIGN.md §2 "bf16 step
# conditioning", profiles/r05_bf16_step_cond.json) are not held to a one-step gradient
# bound: a 2^-9 input perturbation already moves the FP32 step's own gradient by that much.
# They are checked over a 50-step trajectory instead
# (test_config3_bf16_trajectory_matches_fp32).


def _param_groups(model):
    groups = {"encoder": [], "rep_group": [], "item_rep": [], "deconv": []}
    for name, p in model.named_parameters():
        if name.startswith("encoder."):
            groups["encoder"].append(name)
        elif name.startswith("rep_group."):
            groups["rep_group"].append(name)
        elif name == "decoder.item_rep":
            groups["item_rep"].append(name)
        else:
            assert name.startswith("decoder.deconv."), name
            groups["deconv"].append(name)
    return groups


def test_config3_bf16_step_matches_fp32_step(gpu_device, monkeypatch):
    """The benchmarked config-3 step end to end at its size (B = 512): one DPTrainer step
    with amp_dtype=bf16 on a channels-last model with every default fused kernel (MFMA
    deconv forward, small-layer backward, encoder dgrad, fused BN + LeakyReLU, fused
    ReLU) against the fp32 step from the same initial state on the same x and eps
    (reference step: unsupervised.py:108-117 -- loss mean, backward, global-norm clip
    1e-5, Adam lr 1e-3).

    (a) bf16 step vs fp32 step: loss within 1e-2; per parameter group (encoder convs + BN,
        mean / sigma linears, item_rep, deconv stack) the clipped gradients within the bf16
        bound derived above (BF16_STEP_TOL, or BF16_STEP_K times the group's own measured
        sensitivity to a 2^-9 input perturbation of the fp32 step); the Adam update of
        every well-conditioned group points the same way (cosine >= 0.98) and the updated
        parameters agree.
    (b) Inside the bf16 step the SO(3) kernels still compute in fp32: the fused
        exp -> ZYZ -> action launch's output and its gradients (item_rep, v, mu), given the
        step's own inputs and upstream gradient, match the oracle's autograd at fp32 noise
        (1e-5 output per sample with the 2x rule; 1e-4 gradients normwise)."""
    import lie_vae._ops as ops
    from lie_vae.experiments.train_dp import DPTrainer
    from lie_vae.experiments.vae import VAE
    from oracle import lie_ref
    monkeypatch.setattr(torch.backends.cudnn, "deterministic", True)
    monkeypatch.setattr(torch.backends.cudnn, "benchmark", False)
    L, B = 10, 512
    torch.manual_seed(0)
    base = VAE(latent_mode="so3", decoder_mode="action", degrees=L, rep_copies=10, rgb=True,
               batch_norm=True, deconv_hidden=200, mean_mode="s2s2").to(gpu_device)
    base = base.to(memory_format=torch.channels_last)
    groups = _param_groups(base)
    g = torch.Generator().manual_seed(21)
    x = torch.rand(B, 3, 64, 64, generator=g).to(gpu_device)
    eps = torch.randn(1, B, 3, generator=g).to(gpu_device)
    p0 = {k: p.detach().clone() for k, p in base.named_parameters()}
    orig = ops.fused_exp_action
    runs = {}
    xp = x * (1 + 2.0 ** -9 * torch.randn(x.shape, generator=g).to(gpu_device))
    for tag, amp, xin in (("f32", None, x), ("f32_pert", None, xp), ("bf16", torch.bfloat16, x)):
        m = copy.deepcopy(base)
        cap = {}

        def wrap(mu, v, spec, L_, transpose=False, out_dtype=torch.float32, cap=cap):
            out = orig(mu, v, spec, L_, transpose, out_dtype)
            cap["in"] = (mu.detach().clone(), v.detach().clone(), spec.detach().clone())
            cap["out"] = out.detach().clone()
            mu.register_hook(lambda gr: cap.__setitem__("gmu", gr.detach().clone()))
            v.register_hook(lambda gr: cap.__setitem__("gv", gr.detach().clone()))
            out.register_hook(lambda gr: cap.__setitem__("gout", gr.detach().clone()))
            return out
        monkeypatch.setattr(ops, "fused_exp_action", wrap)
        m.decoder.item_rep.register_hook(lambda gr, cap=cap: cap.__setitem__("gF", gr.detach().clone()))
        tr = DPTrainer(m, lr=1e-3, clip_grads=1e-5, amp_dtype=amp)
        loss, _, _ = tr.step(xin, eps)
        torch.cuda.synchronize()
        monkeypatch.setattr(ops, "fused_exp_action", orig)
        assert torch.isfinite(loss)
        named = dict(m.named_parameters())
        runs[tag] = {"loss": float(loss), "cap": cap,
                     "grad": {k: p.grad.detach().float().clone() for k, p in named.items()},
                     "p": {k: p.detach().clone() for k, p in named.items()}}
        del m, tr
    f, fp, b = runs["f32"], runs["f32_pert"], runs["bf16"]
    report = {"loss": abs(b["loss"] - f["loss"]) / abs(f["loss"]),
              "loss_pert": abs(fp["loss"] - f["loss"]) / abs(f["loss"])}

    def cat(d, names):
        return torch.cat([d[n].flatten() for n in names]).double()

    def cos(u, w):
        return float((u @ w) / (u.norm() * w.norm()))
    for gname, names in groups.items():
        gf, gb, gp = cat(f["grad"], names), cat(b["grad"], names), cat(fp["grad"], names)
        df = cat(f["p"], names) - cat(p0, names)
        db = cat(b["p"], names) - cat(p0, names)
        dp = cat(fp["p"], names) - cat(p0, names)
        report[gname] = {"grad": float((gb - gf).norm() / gf.norm()),
                         "kappa": float((gp - gf).norm() / gf.norm()),
                         "update_cos": cos(df, db), "update_cos_pert": cos(df, dp),
                         "param": float((cat(b["p"], names) - cat(f["p"], names)).norm()
                                        / cat(f["p"], names).norm())}
    for gname in groups:
        r = report[gname]
        r["bound"] = max(BF16_STEP_TOL, BF16_STEP_K * r["kappa"])
        r["bound_branch"] = "tol" if r["bound"] == BF16_STEP_TOL else "16kappa"
    print("config3 bf16 vs f32 step:", report)
    # the report is committed (profiles/r05_bf16_step_report.json): which groups passed on
    # which branch of the bound
    out_dir = os.path.join(REPO, "gpurun_out")
    os.makedirs(out_dir, exist_ok=True)
    with open(os.path.join(out_dir, "bf16_step_report.json"), "w") as fh:
        json.dump(report, fh, indent=1, sort_keys=True)
    assert report["loss"] <= 1e-2, report
    for gname in groups:
        r = report[gname]
        bound = r["bound"]
        assert r["grad"] <= bound, (gname, bound, report)
        # the loose branch only for a group whose own fp32 sensitivity is small: a kappa
        # above 0.01 means the fp32 step itself is ill-conditioned there and the one-step
        # bound would say little; those groups are held to the fp32
        # trajectory by test_config3_bf16_trajectory_matches_fp32
        if r["bound_branch"] != "tol" and r["kappa"] > BF16_KAPPA_MAX:
            r["checked_by"] = "trajectory"
        # the Adam update points the same way wherever the gradient is well conditioned
        if bound == BF16_STEP_TOL:
            assert r["update_cos"] >= 0.98, (gname, report)
        assert r["param"] <= 1e-3, (gname, report)
    # (b) the fused SO(3) launch inside the bf16 step against the oracle on its own inputs
    cap = b["cap"]
    mu, v, F = (t.cpu() for t in cap["in"])
    gout = cap["gout"].cpu()
    n = v.shape[0]

    def oracle(dt, grad):
        ts = [t.to(dt).requires_grad_(grad) for t in (mu, v, F)]
        y = lie_ref.block_wigner_apply(lie_ref.mat_to_eazyz(lie_ref.so3_sample(ts[0], ts[1])),
                                       ts[2].expand(n, -1, -1), L)
        if grad:
            (y * gout.to(dt)).sum().backward()
        return y.detach(), [t.grad for t in ts]
    y32, _ = oracle(torch.float32, False)
    y64, (gmu64, gv64, gF64) = oracle(torch.float64, True)
    assert_parity_fp64(host(cap["out"]).reshape(n, -1), y32.numpy().reshape(n, -1),
                       y64.numpy().reshape(n, -1), what="bf16 step: fused SO(3) forward")
    for name, got, ref in (("gF", cap["gF"], gF64), ("gv", cap["gv"], gv64), ("gmu", cap["gmu"], gmu64)):
        assert_normwise(host(got).reshape(1, -1), ref.numpy().reshape(1, -1), 1e-4,
                        what=f"bf16 step: fused SO(3) {name}")


TRAJ_STEPS = 50
TRAJ_COS_MIN = 0.9   # groups on which the fp32 step is stable under a 2^-9 input perturbation
TRAJ_NORM_BAND = 2.0  # the others: bf16's accumulated change within 2x of the scale spread
                      # the perturbed fp32 runs themselves show, either way


def test_config3_bf16_trajectory_matches_fp32(gpu_device, monkeypatch):
    """The bf16 training step against the reference-precision step over a trajectory
    (VERDICT r5 item 6): TRAJ_STEPS DPTrainer steps (unsupervised.py:108-117: loss mean,
    backward, global clip 1e-5, Adam lr 1e-3) from one init on the same seeded batches and
    eps, at config 3 (B = 512, s2s2, l = 10, deconv_hidden 200), in fp32, in fp32 with the
    input perturbed by 2^-9 each step (two noise seeds: the fp32 trajectory's own
    sensitivity), and in bf16 autocast (channels-last, every fused kernel; latent heads in
    fp32, vae.AMP_FP32_HEADS).

    No parameter group is exempted by name; the fp32 runs decide how each is checked.  Per
    group, the accumulated parameter change D_bf16 is compared with D_f32:
      * where the fp32 trajectory is stable (cos(D_pert, D_f32) >= TRAJ_COS_MIN for both
        perturbations; measured: the deconv stack and item_rep, 77% of the parameters),
        cos(D_bf16, D_f32) >= TRAJ_COS_MIN;
      * where it is chaotic (the encoder and the mean / sigma heads: with the reference's
        clip 1e-5 most per-parameter gradients sit near Adam's eps = 1e-8, and a 2^-9 input
        perturbation leaves cos 0.07-0.21 / -0.12-0.66 after 50 fp32 steps,
        profiles/r06_bf16_trajectory_s2s2.json), no run can track the fp32 direction, bf16
        or fp32; the check is that bf16 moves the group on the same scale as fp32 does
        under the perturbation: with s = the perturbed runs' largest max(r, 1/r) of
        r = |D_pert| / |D_f32|, 1/(TRAJ_NORM_BAND s) <= |D_bf16| / |D_f32| <= TRAJ_NORM_BAND s
        (measured: the heads' r reaches 2.9-3.5 in fp32 itself from run to run, bf16 0.6-2.7;
        bf16 rounding noise lifts tiny gradients out of the eps-dominated regime).
    Losses: the mean over the trajectory within 2e-2 relative and within 16x the
    perturbed runs' own difference (the one-step test's 16-kappa factor: bf16 rounds ~80
    times along a gradient path, the perturbation once); every step within 0.25 (the
    chaotic encoder moves the latent rotations: measured up to 0.15, the perturbed fp32
    runs up to 0.05)."""
    import time
    from lie_vae.experiments import vae as vae_mod
    from lie_vae.experiments.train_dp import DPTrainer
    from lie_vae.experiments.vae import VAE
    # MIOpen immediate mode off the packaged find-db, as the benchmarked step runs (its
    # deterministic solvers take ~2 s per step here); the comparison is statistical, so
    # run-to-run summation-order noise is part of what the perturbed runs measure
    monkeypatch.setattr(torch.backends.cudnn, "deterministic", False)
    monkeypatch.setattr(torch.backends.cudnn, "benchmark", False)
    L, B, K = 10, 512, TRAJ_STEPS
    t0 = time.time()
    # fp32 runs NCHW and bf16 channels-last, as bench_train.py runs the two steps (same
    # parameters; only the memory format differs)
    base = VAE(latent_mode="so3", decoder_mode="action", degrees=L, rep_copies=10, rgb=True,
               batch_norm=True, deconv_hidden=200, mean_mode="s2s2").to(gpu_device)
    groups = _param_groups(base)
    p0 = {k: p.detach().clone() for k, p in base.named_parameters()}
    gen = torch.Generator(device=gpu_device).manual_seed(1)
    xs = [torch.rand(B, 3, 64, 64, device=gpu_device, generator=gen) for _ in range(K)]
    es = [torch.randn(1, B, 3, device=gpu_device, generator=gen) for _ in range(K)]

    def noise(seed):
        g = torch.Generator(device=gpu_device).manual_seed(seed)
        return [1 + 2.0 ** -9 * torch.randn(B, 3, 64, 64, device=gpu_device, generator=g) for _ in range(K)]
    runs = {}
    for tag, amp, nz in (("f32", None, None), ("f32_pert", None, noise(2)), ("f32_pert2", None, noise(3)),
                         ("bf16", torch.bfloat16, None)):
        m = copy.deepcopy(base)
        if amp is not None:
            m = m.to(memory_format=torch.channels_last)
        tr = DPTrainer(m, lr=1e-3, clip_grads=1e-5, amp_dtype=amp)
        losses = [tr.step(xs[k] * nz[k] if nz is not None else xs[k], es[k])[0] for k in range(K)]
        torch.cuda.synchronize()
        print(f"trajectory {tag}: {K} steps, {time.time() - t0:.1f} s", flush=True)
        named = dict(m.named_parameters())
        runs[tag] = {"loss": [float(x) for x in losses],
                     "delta": {g: torch.cat([(named[n].detach() - p0[n]).flatten() for n in names]).double()
                               for g, names in groups.items()}}
        del m, tr, nz
    f = runs["f32"]
    rep = {"steps": K, "amp_fp32_heads": vae_mod.AMP_FP32_HEADS,
           "params": {g: int(sum(base.get_parameter(n).numel() for n in names)) for g, names in groups.items()}}
    for tag in ("f32_pert", "f32_pert2", "bf16"):
        o = runs[tag]
        rel = [abs(x - y) / abs(y) for x, y in zip(o["loss"], f["loss"])]
        rep[tag] = {"loss_rel_max": max(rel), "loss_mean_rel": abs(sum(o["loss"]) - sum(f["loss"])) / sum(f["loss"])}
        for g in groups:
            u, w = o["delta"][g], f["delta"][g]
            rep[tag][g] = {"cos": float(u @ w / (u.norm() * w.norm())), "rel": float((u - w).norm() / w.norm()),
                           "norm_ratio": float(u.norm() / w.norm())}
    print("config3 bf16 vs f32 trajectory:", json.dumps(rep))
    out_dir = os.path.join(REPO, "gpurun_out")
    os.makedirs(out_dir, exist_ok=True)
    with open(os.path.join(out_dir, "bf16_trajectory_report.json"), "w") as fh:
        json.dump(dict(rep, loss_f32=f["loss"], loss_bf16=runs["bf16"]["loss"]), fh, indent=1)
    pert_mean = max(rep[t]["loss_mean_rel"] for t in ("f32_pert", "f32_pert2"))
    assert rep["bf16"]["loss_mean_rel"] <= min(2e-2, max(1e-3, 16 * pert_mean)), rep
    assert rep["bf16"]["loss_rel_max"] <= 0.25, rep
    stable = [g for g in groups if min(rep[t][g]["cos"] for t in ("f32_pert", "f32_pert2")) >= TRAJ_COS_MIN]
    rep["stable_groups"] = stable
    # the decoder (most of the parameters) must be among the stable groups
    assert "deconv" in stable and "item_rep" in stable, rep
    for g in groups:
        if g in stable:
            assert rep["bf16"][g]["cos"] >= TRAJ_COS_MIN, (g, rep)
        else:
            spread = max(max(rep[t][g]["norm_ratio"], 1 / rep[t][g]["norm_ratio"]) for t in ("f32_pert", "f32_pert2"))
            band = TRAJ_NORM_BAND * spread
            assert 1 / band <= rep["bf16"][g]["norm_ratio"] <= band, (g, band, rep)


def test_config3_iwae_n500_vs_oracle(gpu_device):
    """The reference's evaluation (main.py:134-139): IWAE log-likelihood with n = 500 on
    the conv VAE, one image per call.  The SO(3) terms (log q over the 500 samples, the
    fused decode) against the oracle fed the GPU encoder features and the same eps; the
    recon term from the GPU deconv output (MIOpen vs CPU is checked in the config-3 test).
    A 2-image call gives the mean of the two 1-image calls (same eps slices)."""
    from lie_vae.experiments.vae import VAE
    from oracle import lie_ref
    L, C, n = 10, 10, 500
    torch.manual_seed(5)
    cpu = VAE(latent_mode="so3", decoder_mode="action", degrees=L, rep_copies=C, rgb=True,
              batch_norm=True, deconv_hidden=200, mean_mode="s2s2").eval()
    gvae = copy.deepcopy(cpu).to(gpu_device).eval()
    g = torch.Generator().manual_seed(6)
    x = torch.rand(2, 3, 64, 64, generator=g)
    eps = torch.randn(n, 2, 3, generator=g)
    lls = []
    rep = cpu.rep_group
    for b in range(2):
        cap = {}
        hooks = [_capture(gvae.encoder, cap, "enc"), _capture(gvae.decoder.deconv, cap, "dec")]
        with torch.no_grad():
            ll = gvae.log_likelihood(x[b:b + 1].to(gpu_device), n=n,
                                     eps=eps[:, b:b + 1].to(gpu_device))
        for h in hooks:
            h.remove()
        lls.append(float(ll))
        h_gpu, xr_gpu = cap["enc"][1].cpu(), cap["dec"][1].cpu()
        with torch.no_grad():
            sig = lie_ref.n0_sigma(rep.reparameterize.sigma_linear(h_gpu))
            vv = lie_ref.n0_sample(sig, eps[:, b:b + 1])
            lq = lie_ref.so3_log_posterior(vv, sig, 10)                      # (n, 1)
        rec = ((xr_gpu.reshape(n, 1, 3, 64, 64) - x[b:b + 1]) ** 2).sum((-1, -2, -3))
        w = (-rec - math.log(8 * math.pi ** 2) - lq).double()
        ll_ref = float((torch.logsumexp(w, 0) - math.log(n)).mean())
        assert ll_ref == pytest.approx(lls[-1], rel=1e-5)
    with torch.no_grad():
        ll2 = gvae.log_likelihood(x.to(gpu_device), n=n, eps=eps.to(gpu_device))
    assert float(ll2) == pytest.approx(sum(lls) / 2, rel=1e-5)


def test_dp_trainer_graph_replay_matches_eager(gpu_device):
    """DPTrainer.capture: the whole step (forward, backward, all-reduce, clip, capturable
    Adam) as one hipGraph.  Its warm-up is undone, so replays from a model's state follow
    the same trajectory as eager steps from a copy of that state (MIOpen pinned
    deterministic; eps injected)."""
    from lie_vae.experiments.train_dp import DPTrainer
    from lie_vae.experiments.vae import VAE
    det, bench = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    try:
        torch.manual_seed(0)
        base = VAE(latent_mode="so3", decoder_mode="action", degrees=10, rep_copies=10,
                   rgb=True, batch_norm=True, deconv_hidden=200,
                   mean_mode="s2s2").to(gpu_device)
        g = torch.Generator().manual_seed(4)
        xs = [torch.rand(64, 3, 64, 64, generator=g).to(gpu_device) for _ in range(4)]
        eps = [torch.randn(1, 64, 3, generator=g).to(gpu_device) for _ in range(4)]
        me, mg = copy.deepcopy(base), copy.deepcopy(base)
        te = DPTrainer(me, lr=1e-3, clip_grads=1e-5, graph=True)
        tg = DPTrainer(mg, lr=1e-3, clip_grads=1e-5, graph=True)
        # one eager step first (Adam state exists, the model holds a live autograd graph)
        te.step(xs[0], eps[0])
        tg.step(xs[0], eps[0])
        replay = tg.capture(xs[1], eps[1])
        for x, e in zip(xs[1:], eps[1:]):
            le = [float(t.double().mean()) for t in te.step(x, e)]
            lg = [float(t.double().mean()) for t in replay(x, e)]
            torch.cuda.synchronize()
            assert le == pytest.approx(lg, rel=1e-5)
        pe = torch.cat([p.detach().flatten() for p in me.parameters()])
        pg = torch.cat([p.detach().flatten() for p in mg.parameters()])
        torch.testing.assert_close(pg, pe, rtol=1e-4, atol=1e-6)
        be = torch.cat([b.double().flatten() for b in me.buffers()])
        bg = torch.cat([b.double().flatten() for b in mg.buffers()])
        torch.testing.assert_close(bg, be, rtol=1e-4, atol=1e-6)
    finally:
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = det, bench


_DP2_WORKER = r"""
import os, sys
import numpy as np
import torch
import torch.distributed as dist
sys.path[:0] = [sys.argv[1]]
from lie_vae.experiments.train_dp import DPTrainer
from lie_vae.experiments.vae import VAE
PER_RANK = int(sys.argv[3])
dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
torch.backends.cudnn.benchmark = False
torch.backends.cudnn.deterministic = True     # MIOpen: deterministic solutions


def model():
    torch.manual_seed(0)
    return VAE(latent_mode="so3", decoder_mode="action", degrees=10, rep_copies=10, rgb=True,
               batch_norm=True, deconv_hidden=200, mean_mode="s2s2").to(dev)


def flat(ps, grad=False):
    return torch.cat([(q.grad if grad else q.detach()).flatten() for q in ps]).cpu()


g = torch.Generator().manual_seed(100)          # the global batch; rank r takes shard r
xs = [torch.rand(world * PER_RANK, 3, 64, 64, generator=g) for _ in range(2)]
es = [torch.randn(1, world * PER_RANK, 3, generator=g) for _ in range(2)]
sh = slice(rank * PER_RANK, (rank + 1) * PER_RANK)
m = model()
tr = DPTrainer(m, lr=1e-3, clip_grads=1e-5, sync_bn=True)
names = [n for n, _ in m.named_parameters()]
res = {"sizes": np.array([q.numel() for q in m.parameters()])}
for it in range(2):
    if rank == 0:
        # the single-device step's gradient on the concatenated batch AT THE REPLICAS'
        # CURRENT PARAMETERS (unsupervised.py:108-116: loss mean, backward, global clip),
        # plain BatchNorm, no collective
        ref = model()
        ref.load_state_dict(m.state_dict())
        recon, kl, _ = ref.elbo(xs[it].to(dev), 1, eps=es[it].to(dev))
        lref = (recon + kl).mean()
        lref.backward()
        torch.nn.utils.clip_grad_norm_(ref.parameters(), 1e-5)
        res[f"at_grad{it}"] = flat(ref.parameters(), True).numpy()
        res[f"at_loss{it}"] = np.array([float(lref)])
        del ref
    l, _, _ = tr.step(xs[it][sh].to(dev), es[it][:, sh].to(dev))
    torch.cuda.synchronize()
    for name, t in (("grad", flat(m.parameters(), True)), ("p", flat(m.parameters())),
                    ("loss", l.double().reshape(1).cpu())):
        ts = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(ts, t)
        res[f"{name}{it}"] = torch.stack(ts).numpy()
dist.destroy_process_group()
if rank == 0:
    # the single-device trajectory: two reference steps on the concatenated batches from
    # the same initial state
    m1 = model()
    t1 = DPTrainer(m1, lr=1e-3, clip_grads=1e-5)
    for it in range(2):
        t1.step(xs[it].to(dev), es[it].to(dev))
        torch.cuda.synchronize()
        res[f"ref_p{it}"] = flat(m1.parameters()).numpy()
    np.savez(sys.argv[2], names=np.array(names), **res)
"""


def _worst_tensors(err, sizes, names, k=3):
    offs = np.concatenate([[0], np.cumsum(sizes)])
    per = [(float(np.linalg.norm(err[offs[i]:offs[i + 1]])), str(names[i]))
           for i in range(len(sizes))]
    return sorted(per, reverse=True)[:k]


def test_config4_dp_two_ranks_share_one_gpu(tmp_path):
    """Config 4's data-parallel step at its per-GPU shard (512 images per rank) with two
    rank processes on the one GPU of the box (gloo carries the bucketed gradient all-reduce
    and the SyncBatchNorm moments; RCCL refuses two ranks per device), against the
    single-device step on the concatenated 1,024-image batch (unsupervised.py:108-117 on
    one device, main.py:17), MIOpen pinned deterministic:
      * the replicas stay bit-identical over two steps, and the ranks saw different data;
      * at each step the all-reduced, globally clipped gradient equals the single-device
        gradient at the same parameters to fp32 summation noise (normwise), and the global
        loss is the mean of the ranks' losses.  The encoder's gradients pass through the
        BatchNorm backward, where SyncBatchNorm's moments (gathered per-rank counts) and
        BatchNorm's one-pass moments round differently and the mean subtraction amplifies
        it (measured 0.9-1.4e-4 normwise): 1e-3 there; 1e-5 for every other parameter (measured
        1.6e-6);
      * two DP steps land on the single-device trajectory from the same initial state."""
    import os
    import socket
    import subprocess
    import sys
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "dp2_worker.py"
    script.write_text(_DP2_WORKER)
    out = tmp_path / "dp2.npz"
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                    "--nproc-per-node=2", "--master-addr=127.0.0.1", f"--master-port={port}",
                    str(script), os.path.join(repo, "lie-vae_amd"), str(out), "512"],
                   env=env, check=True, timeout=300)
    r = np.load(out)
    sizes, names = r["sizes"], r["names"]
    report = []
    for it in range(2):
        p, grad, loss = r[f"p{it}"], r[f"grad{it}"], r[f"loss{it}"]
        assert np.isfinite(p).all() and np.isfinite(grad).all() and np.isfinite(loss).all()
        assert np.array_equal(p[0], p[1]), f"replicas diverged at step {it + 1}"
        assert np.array_equal(grad[0], grad[1])
        assert loss[0, 0] != loss[1, 0]  # different shards
        assert loss.mean() == pytest.approx(float(r[f"at_loss{it}"][0]), rel=1e-5)
        rg = r[f"at_grad{it}"]
        err = np.linalg.norm(grad[0] - rg) / np.linalg.norm(rg)
        # parameters whose gradient does not pass through a BatchNorm backward
        rest = np.concatenate([np.full(n, not str(nm).startswith("encoder."))
                               for n, nm in zip(sizes, names)])
        err_rest = np.linalg.norm((grad[0] - rg)[rest]) / np.linalg.norm(rg[rest])
        perr = np.linalg.norm(p[0] - r[f"ref_p{it}"]) / np.linalg.norm(r[f"ref_p{it}"])
        report.append((it + 1, err, err_rest, perr, _worst_tensors(grad[0] - rg, sizes, names)))
    print(report)
    for step, err, err_rest, perr, worst in report:
        assert err_rest <= 1e-5, f"step {step}: non-encoder gradient vs single device {err_rest:.2e}"
        assert err <= 1e-3, f"step {step}: gradient vs single device {err:.2e}; {worst}"
        assert perr <= 1e-4, f"step {step}: parameters vs single-device trajectory {perr:.2e}"


_DP2_BF16_WORKER = r"""
import os, sys
import numpy as np
import torch
import torch.distributed as dist
sys.path[:0] = [sys.argv[1]]
from lie_vae.experiments.train_dp import DPTrainer
from lie_vae.experiments.vae import VAE
PER_RANK = int(sys.argv[3])
dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
solo = [dist.new_group([r]) for r in range(world)]   # every rank creates every group
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
torch.backends.cudnn.benchmark = False
torch.backends.cudnn.deterministic = True


def model():
    torch.manual_seed(0)
    return VAE(latent_mode="so3", decoder_mode="action", degrees=10, rep_copies=10, rgb=True,
               batch_norm=True, deconv_hidden=200,
               mean_mode="s2s2").to(dev).to(memory_format=torch.channels_last)


def flat_grad(m):
    return torch.cat([q.grad.detach().flatten() for q in m.parameters()]).cpu()


g = torch.Generator().manual_seed(300)
xs = [torch.rand(world * PER_RANK, 3, 64, 64, generator=g) for _ in range(2)]
es = [torch.randn(1, world * PER_RANK, 3, generator=g) for _ in range(2)]
sh = slice(rank * PER_RANK, (rank + 1) * PER_RANK)
m = model()
# clip off: the bucket then holds exactly the mean of the ranks' local gradients
tr = DPTrainer(m, lr=1e-3, clip_grads=0, amp_dtype=torch.bfloat16)
res = {}
for it in range(2):
    # this rank's LOCAL bf16 gradient at the replicas' current parameters: a one-rank
    # trainer (its own group) on the same shard, same kernels, same cached bf16 copies path
    loc = model()
    loc.load_state_dict(m.state_dict())
    tl = DPTrainer(loc, lr=1e-3, clip_grads=0, amp_dtype=torch.bfloat16, group=solo[rank],
                   broadcast=False)
    tl.ar.zero_grad()
    lo, _, _ = tl.loss(xs[it][sh].to(dev), es[it][:, sh].to(dev), 1.0)
    lo.backward()
    tl.ar.finish()
    torch.cuda.synchronize()
    gl = flat_grad(loc)
    del loc, tl
    tr.step(xs[it][sh].to(dev), es[it][:, sh].to(dev))
    torch.cuda.synchronize()
    gd = flat_grad(m)
    for name, t in (("local", gl), ("dp", gd)):
        ts = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(ts, t)
        res[f"{name}{it}"] = torch.stack(ts).numpy()
dist.destroy_process_group()
if rank == 0:
    np.savez(sys.argv[2], **res)
"""


def test_config4_dp_bf16_bucket_sums_two_ranks(tmp_path):
    """ADVICE r4 (nets._CachedCast / BucketedAllReduce): the bf16 DP step with the cached
    bf16 parameter copies, whose backward adds straight into the gradient buckets, over two
    rank processes on the box's one GPU (gloo all-reduce), two steps.  With clipping off the
    all-reduced bucket must equal the mean of the two ranks' LOCAL bf16 gradients computed
    at the same parameters on the same shards (bit for bit: same kernels, deterministic
    MIOpen, the same fp32 (a + b) / 2) -- a bucket launched before all of its gradients
    landed would miss some -- and the replicas stay identical."""
    import socket
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "dp2_bf16_worker.py"
    script.write_text(_DP2_BF16_WORKER)
    out = tmp_path / "dp2_bf16.npz"
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                    "--nproc-per-node=2", "--master-addr=127.0.0.1", f"--master-port={port}",
                    str(script), os.path.join(repo, "lie-vae_amd"), str(out), "128"],
                   env=env, check=True, timeout=300)
    r = np.load(out)
    for it in range(2):
        loc, dp = r[f"local{it}"], r[f"dp{it}"]
        assert np.isfinite(dp).all()
        assert np.array_equal(dp[0], dp[1]), f"replicas' gradients differ at step {it + 1}"
        want = (loc[0] + loc[1]) / np.float32(2)
        err = np.abs(dp[0] - want).max() / np.abs(want).max()
        assert err <= 1e-6, f"step {it + 1}: bucket vs mean of local gradients {err:.2e}"


# ----------------------------------------------- decoder ConvTranspose2d on MFMA (§8 f1)
@pytest.mark.parametrize("N,Cin,Cout,H,W", [(3, 200, 200, 16, 16), (4, 200, 200, 4, 4),
                                           (2, 16, 8, 5, 3), (5, 64, 200, 7, 9),
                                           (3, 200, 3, 32, 32), (2, 40, 1, 9, 21),
                                           (2, 200, 4, 17, 16)])
def test_mfma_deconv_matches_conv_transpose(gpu_device, N, Cin, Cout, H, W):
    """lv_deconv4s2_fwd_bf16 (csrc/deconv.hip: four sub-pixel implicit GEMMs on
    v_mfma_f32_16x16x32_bf16) and, for Cout <= 4, lv_deconv4s2_small_fwd_bf16 (one quad GEMM
    over the 3x3 neighbourhood) against conv_transpose2d(stride 2, padding 1) evaluated in
    float64 on the same bf16 operands: fp32 accumulation, one bf16 rounding of the output
    (|err| <= 2^-8 |ref| + 1e-3 rms(ref)); ragged pixel tiles, border taps, small C."""
    from lie_vae.experiments.nets import _Deconv4s2
    g = torch.Generator().manual_seed(N * 1000 + Cin + H)
    x = torch.randn(N, Cin, H, W, generator=g).to(torch.bfloat16)
    w = (torch.randn(Cin, Cout, 4, 4, generator=g) * 0.05).to(torch.bfloat16)
    b = torch.randn(Cout, generator=g)
    ref = torch.nn.functional.conv_transpose2d(x.double(), w.double(), b.double(), 2, 1)
    y = _Deconv4s2.apply(x.to(gpu_device).contiguous(memory_format=torch.channels_last),
                         w.to(gpu_device), b.to(gpu_device))
    assert y.shape == ref.shape and y.dtype == torch.bfloat16
    assert y.is_contiguous(memory_format=torch.channels_last)
    yd = y.double().cpu()
    rms = ref.square().mean().sqrt()
    bad = (yd - ref).abs() > 2.0 ** -8 * ref.abs() + 1e-3 * rms
    assert not bad.any(), f"{int(bad.sum())} elements off, max err {(yd - ref).abs().max():.3e}"


def test_mfma_deconv_module_under_autocast(gpu_device):
    """MfmaConvTranspose2d (nets.MFMA_DECONV) in a bf16 autocast region on channels-last
    input: forward within bf16 rounding of nn.ConvTranspose2d's, and the backward (aten
    convolution_backward on the same bf16 operands) gives the plain layer's gradients."""
    from lie_vae.experiments.nets import MfmaConvTranspose2d
    torch.manual_seed(9)
    m = MfmaConvTranspose2d(200, 200, 4, 2, 1).to(gpu_device).to(memory_format=torch.channels_last)
    r = torch.nn.ConvTranspose2d(200, 200, 4, 2, 1).to(gpu_device).to(memory_format=torch.channels_last)
    r.load_state_dict(m.state_dict())
    x = torch.randn(8, 200, 8, 8, device=gpu_device).contiguous(memory_format=torch.channels_last)
    gy = torch.randn(8, 200, 16, 16, device=gpu_device)
    xs = [x.clone().requires_grad_(True) for _ in range(2)]
    with torch.autocast("cuda", dtype=torch.bfloat16):
        ym, yr = m(xs[0]), r(xs[1])
    assert ym.dtype == yr.dtype == torch.bfloat16
    torch.testing.assert_close(ym.float(), yr.float(), rtol=2e-2, atol=2e-2)
    (ym.float() * gy).sum().backward()
    (yr.float() * gy).sum().backward()
    torch.testing.assert_close(xs[0].grad, xs[1].grad, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(m.weight.grad, r.weight.grad, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(m.bias.grad, r.bias.grad, rtol=2e-2, atol=2e-2)


def F32_ACC_TOL(K):
    """Max-error allowance (relative to the output's scale) for a K-term fp32 accumulation:
    sqrt(K) units of 2^-23, the random-walk size of K fp32 roundings with a 2x margin.  Used
    where the MFMA kernel's sequential K order and MIOpen's blocked order differ (MIOpen can
    be the more accurate at large K)."""
    return K ** 0.5 * 2.0 ** -23


@pytest.mark.parametrize("N,Cin,Cout,H,W,relu", [(3, 200, 200, 16, 16, 0), (4, 200, 200, 4, 4, 1),
                                                (2, 16, 8, 5, 3, 0), (5, 64, 200, 7, 9, 1),
                                                (2, 200, 5, 17, 16, 0), (2, 12, 208, 6, 10, 0),
                                                (64, 200, 200, 8, 8, 1)])
def test_mfma_deconv_f32_matches_float64(gpu_device, N, Cin, Cout, H, W, relu):
    """lv_deconv4s2_fwd_f32 (fp32 operands on v_mfma_f32_16x16x4_f32, NCHW output) against
    conv_transpose2d(stride 2, padding 1) in float64 on the same fp32 operands.  The bar is
    the reference's own precision: torch's fp32 layer (MIOpen, what nn.ConvTranspose2d runs
    in the reference's fp32 training) has some max error e against float64; ours must stay
    within 2 e (or F32_ACC_TOL(K) of the output's scale), and within 1e-5 normwise.  Ragged pixel
    tiles, border taps, Cout not a multiple of 16, the fused ReLU; the channels-last twin
    output bit for bit equal to y."""
    from lie_vae.experiments.nets import _Deconv4s2F32
    from lie_vae import _lib
    g = torch.Generator().manual_seed(N * 1000 + Cin + H + Cout)
    x = torch.randn(N, Cin, H, W, generator=g)
    w = torch.randn(Cin, Cout, 4, 4, generator=g) * 0.05
    b = torch.randn(Cout, generator=g)
    ref = torch.nn.functional.conv_transpose2d(x.double(), w.double(), b.double(), 2, 1)
    xg, wg, bg = x.to(gpu_device), w.to(gpu_device), b.to(gpu_device)
    yt = torch.nn.functional.conv_transpose2d(xg, wg, bg, 2, 1)
    if relu:
        ref, yt = ref.clamp_min(0), yt.clamp_min(0)
    twin = Cout % 4 == 0
    y, ycl = _Deconv4s2F32.apply(xg, wg, bg, _lib.LV_DECONV_RELU_OUT if relu else 0, None, twin)
    assert y.shape == ref.shape and y.dtype == torch.float32 and y.is_contiguous()
    if twin:  # the channels-last copy the epilogue writes beside y (the next layer's input)
        assert ycl.is_contiguous(memory_format=torch.channels_last) and torch.equal(ycl, y)
    yd, ytd = y.double().cpu(), yt.double().cpu()
    e, e_t = (yd - ref).abs().max().item(), (ytd - ref).abs().max().item()
    scale = ref.abs().max().item()
    assert e <= max(2 * e_t, F32_ACC_TOL(4 * Cin) * scale), (e, e_t, scale)
    assert (yd - ref).norm() <= 1e-5 * ref.norm(), ((yd - ref).norm() / ref.norm()).item()


def test_mfma_deconv_f32_module_matches_plain_layer(gpu_device):
    """MfmaConvTranspose2d in fp32 (no autocast; nets.MFMA_DECONV_F32) with the fused ReLU:
    forward within fp32 rounding of nn.ConvTranspose2d + ReLU, gradients (the same
    convolution_backward, gy masked by the ReLU) likewise; a second layer reading the
    first's channels-last twin gives the same bits as reading a transposed copy."""
    from lie_vae.experiments.nets import MfmaConvTranspose2d
    torch.manual_seed(19)
    m = MfmaConvTranspose2d(200, 200, 4, 2, 1).to(gpu_device)
    m.relu_out = True
    m.cl_twin_out = True
    m2 = MfmaConvTranspose2d(200, 200, 4, 2, 1).to(gpu_device)
    with torch.no_grad():
        y1 = m(torch.randn(4, 200, 4, 4, device=gpu_device))
        assert y1._lv_cl_twin[0] is not None
        z_twin = m2(y1)
        z_copy = m2(y1.clone())
    assert torch.equal(z_twin, z_copy)
    m.cl_twin_out = False
    r = torch.nn.ConvTranspose2d(200, 200, 4, 2, 1).to(gpu_device)
    r.load_state_dict(m.state_dict())
    x = torch.randn(16, 200, 8, 8, device=gpu_device)
    gy = torch.randn(16, 200, 16, 16, device=gpu_device)
    xs = [x.clone().requires_grad_(True) for _ in range(2)]
    ym, yr = m(xs[0]), torch.relu(r(xs[1]))
    torch.testing.assert_close(ym, yr, rtol=1e-5, atol=1e-5)
    (ym * gy).sum().backward()
    (yr * gy).sum().backward()
    torch.testing.assert_close(xs[0].grad, xs[1].grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(m.weight.grad, r.weight.grad, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(m.bias.grad, r.bias.grad, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("N,Cin,Cout,H,W", [(3, 200, 3, 32, 32), (2, 40, 1, 9, 21), (2, 200, 4, 17, 16),
                                           (1, 248, 3, 5, 40), (2, 64, 200, 7, 9)])
def test_mfma_deconv_backward_matches_autograd(gpu_device, N, Cin, Cout, H, W):
    """_Deconv4s2.backward: for Cout <= 4 lv_deconv4s2_small_bwd_bf16 (dgrad, wgrad and
    bias from the quad view; csrc/deconv.hip), otherwise MIOpen's gx/gw with the library's
    per-channel bias sum (lv_channel_sum_bf16) -- against float64 autograd of
    conv_transpose2d on the same bf16-rounded x, w and gy.  Tolerance: the library's gx, gw
    are rounded to bf16 once (|err| <= 2^-8 |ref| + 1e-3 rms); MIOpen's (Cout > 4) measure up
    to ~2% off (its bf16 split-K partials), checked at 2^-5 |ref| + 1e-2 rms; gb is fp32
    (1e-4 relative + 1e-5 rms)."""
    from lie_vae.experiments.nets import _Deconv4s2
    g = torch.Generator().manual_seed(N * 7 + Cin + Cout + H * W)
    x = torch.randn(N, Cin, H, W, generator=g).to(torch.bfloat16)
    w = (torch.randn(Cin, Cout, 4, 4, generator=g) * 0.05).to(torch.bfloat16)
    b = torch.randn(Cout, generator=g)
    gy = torch.randn(N, Cout, 2 * H, 2 * W, generator=g).to(torch.bfloat16)
    xr, wr, br = (t.double().requires_grad_(True) for t in (x, w, b))
    torch.nn.functional.conv_transpose2d(xr, wr, br, 2, 1).backward(gy.double())
    xd = x.to(gpu_device).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    wd = w.to(gpu_device).requires_grad_(True)
    bd = b.to(gpu_device).requires_grad_(True)
    _Deconv4s2.apply(xd, wd, bd).backward(gy.to(gpu_device).contiguous(memory_format=torch.channels_last))
    rel_l, abs_l = (2.0 ** -8, 1e-3) if Cout <= 4 else (2.0 ** -5, 1e-2)
    for name, got, ref, rel, absr in (("gx", xd.grad, xr.grad, rel_l, abs_l),
                                      ("gw", wd.grad, wr.grad, rel_l, abs_l),
                                      ("gb", bd.grad, br.grad, 1e-4, 1e-5)):
        assert got.shape == ref.shape, name
        gd = got.double().cpu()
        rms = ref.square().mean().sqrt()
        bad = (gd - ref).abs() > rel * ref.abs() + absr * rms
        assert not bad.any(), f"{name}: {int(bad.sum())} of {bad.numel()} off, max err {(gd - ref).abs().max():.3e}"


@pytest.mark.parametrize("N,Cin,Cout,H,W", [(3, 100, 200, 16, 16), (2, 200, 400, 8, 8), (2, 48, 96, 10, 6)])
def test_mfma_conv_dgrad_matches_autograd(gpu_device, N, Cin, Cout, H, W):
    """MfmaDgradConv2d (the encoder's Conv2d(c, 2c, 4, 2, 1)): gx from
    lv_deconv4s2_fwd_bf16 with the Conv2d weight read as a transposed-convolution weight,
    against float64 autograd of conv2d on the same bf16 x, w and gy (fp32 accumulation,
    one bf16 rounding: 2^-8 |ref| + 1e-3 rms); forward and gw / gb are MIOpen's (2^-5 |ref|
    + 1e-2 rms, as in test_mfma_deconv_backward_matches_autograd)."""
    from lie_vae.experiments.nets import _Conv4s2
    g = torch.Generator().manual_seed(N * 11 + Cin + H)
    x = torch.randn(N, Cin, H, W, generator=g).to(torch.bfloat16)
    w = (torch.randn(Cout, Cin, 4, 4, generator=g) * 0.05).to(torch.bfloat16)
    b = torch.randn(Cout, generator=g).to(torch.bfloat16)
    gy = torch.randn(N, Cout, H // 2, W // 2, generator=g).to(torch.bfloat16)
    xr, wr, br = (t.double().requires_grad_(True) for t in (x, w, b))
    torch.nn.functional.conv2d(xr, wr, br, 2, 1).backward(gy.double())
    xd = x.to(gpu_device).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    wd = w.to(gpu_device).requires_grad_(True)
    bd = b.to(gpu_device).requires_grad_(True)
    _Conv4s2.apply(xd, wd, bd).backward(gy.to(gpu_device).contiguous(memory_format=torch.channels_last))
    for name, got, ref, rel, absr in (("gx", xd.grad, xr.grad, 2.0 ** -8, 1e-3),
                                      ("gw", wd.grad, wr.grad, 2.0 ** -5, 1e-2),
                                      ("gb", bd.grad, br.grad, 2.0 ** -5, 1e-2)):
        assert got.shape == ref.shape, name
        gd = got.double().cpu()
        rms = ref.square().mean().sqrt()
        bad = (gd - ref).abs() > rel * ref.abs() + absr * rms
        assert not bad.any(), f"{name}: {int(bad.sum())} of {bad.numel()} off, max err {(gd - ref).abs().max():.3e}"


@pytest.mark.parametrize("N,Cin,Cout,H,W", [(3, 200, 400, 8, 8), (2, 120, 36, 10, 6)])
def test_mfma_conv_dgrad_f32_matches_float64(gpu_device, N, Cin, Cout, H, W):
    """The fp32 encoder dgrad (_Conv4s2F32: gx by lv_deconv4s2_fwd_f32 with the Conv2d weight
    read as a transposed-convolution weight) against float64 autograd of conv2d on the same
    fp32 x, w and gy: within 2x torch's own fp32 gx error (MIOpen, the reference's layer) or
    F32_ACC_TOL(K) of the scale, 1e-5 normwise; gw / gb are MIOpen's own (fp32 tolerance)."""
    from lie_vae.experiments.nets import _Conv4s2F32
    g = torch.Generator().manual_seed(N * 13 + Cin + H)
    x = torch.randn(N, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, 4, 4, generator=g) * 0.05
    b = torch.randn(Cout, generator=g)
    gy = torch.randn(N, Cout, H // 2, W // 2, generator=g)
    xr, wr, br = (t.double().requires_grad_(True) for t in (x, w, b))
    torch.nn.functional.conv2d(xr, wr, br, 2, 1).backward(gy.double())
    xd, wd, bd = (t.to(gpu_device).requires_grad_(True) for t in (x, w, b))
    _Conv4s2F32.apply(xd, wd, bd).backward(gy.to(gpu_device))
    xt = x.to(gpu_device).requires_grad_(True)
    torch.nn.functional.conv2d(xt, w.to(gpu_device), b.to(gpu_device), 2, 1).backward(gy.to(gpu_device))
    ref = xr.grad
    e = (xd.grad.double().cpu() - ref).abs().max().item()
    e_t = (xt.grad.double().cpu() - ref).abs().max().item()
    assert e <= max(2 * e_t, F32_ACC_TOL(4 * Cout) * ref.abs().max().item()), (e, e_t)
    assert (xd.grad.double().cpu() - ref).norm() <= 1e-5 * ref.norm()
    torch.testing.assert_close(wd.grad.double().cpu(), wr.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(bd.grad.double().cpu(), br.grad, rtol=1e-4, atol=1e-4)


def test_small_deconv_mask_gx_bitwise(gpu_device):
    """The RGB layer's LV_DECONV_MASK_GX (dgrad's epilogue masks gx by x > 0, x being a ReLU
    output) against the plain kernels followed by aten's threshold_backward: bit for bit."""
    from lie_vae import _lib
    from lie_vae.experiments.nets import _Deconv4s2
    g = torch.Generator().manual_seed(17)
    x = torch.randn(3, 200, 17, 16, generator=g).to(torch.bfloat16).to(gpu_device)
    x = torch.relu(x).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(200, 3, 4, 4, generator=g) * 0.05).to(torch.bfloat16).to(gpu_device)
    b = torch.randn(3, generator=g).to(gpu_device)
    gy = torch.randn(3, 3, 34, 32, generator=g).to(torch.bfloat16).to(gpu_device)
    gy = gy.contiguous(memory_format=torch.channels_last)
    res = {}
    for tag, flags in (("ref", 0), ("mask", _lib.LV_DECONV_MASK_GX)):
        xi = x.detach().clone().requires_grad_(True)
        wi, bi = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
        y = _Deconv4s2.apply(xi, wi, bi, flags)
        y.backward(gy)
        gx = xi.grad
        if tag == "ref":
            gx = torch.ops.aten.threshold_backward(gx, x, 0)
        res[tag] = (y.detach(), gx, wi.grad, bi.grad)
    for name, a, r in zip(("y", "gx", "gw", "gb"), res["mask"], res["ref"]):
        assert torch.equal(a, r), f"mask: {name}"


def test_fused_layers_fall_back_outside_their_contract(gpu_device):
    """FusedBatchNormLeakyReLU with bf16 parameters (model.to(bfloat16)) or a 16-byte
    misaligned input takes the BatchNorm2d + leaky_relu fallback (the kernels read fp32
    gamma / beta / running stats and load x in 16-byte pieces); an RGB deconv layer with
    Cin = 256 (> the small-Cout backward's 248-channel bound) runs nn.ConvTranspose2d
    instead of failing in backward."""
    from lie_vae.experiments.nets import FusedBatchNormLeakyReLU, MfmaConvTranspose2d
    m = FusedBatchNormLeakyReLU(64, 0.2).to(gpu_device)
    x = torch.randn(8, 64, 8, 8, device=gpu_device).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    assert m._fused_ok(x)
    assert not copy.deepcopy(m).to(torch.bfloat16)._fused_ok(x)
    buf = torch.empty(8 * 64 * 8 * 8 + 8, device=gpu_device, dtype=torch.bfloat16)
    xm = buf[1:1 + x.numel()].view(8, 8, 8, 64).permute(0, 3, 1, 2)  # channels-last, +2 bytes
    assert xm.data_ptr() % 16 and not m._fused_ok(xm)
    mb = copy.deepcopy(m).to(torch.bfloat16)
    y = mb(x.requires_grad_(True))
    y.float().sum().backward()
    assert torch.isfinite(x.grad.float()).all() and mb.weight.grad.dtype == torch.bfloat16
    big = MfmaConvTranspose2d(256, 3, 4, 2, 1).to(gpu_device).to(memory_format=torch.channels_last)
    xb = torch.randn(2, 256, 8, 8, device=gpu_device).contiguous(memory_format=torch.channels_last)
    assert not big._mfma_ok(xb)
    xb.requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        yb = big(xb)
    yb.float().sum().backward()
    assert torch.isfinite(xb.grad).all() and big.weight.grad is not None


def test_fused_relu_deconvnet_bitwise(gpu_device, monkeypatch):
    """DeconvNet with its ReLUs fused into the MFMA layers (nets.FUSED_RELU: relu_out on the
    2nd / 3rd / 4th layers' forward epilogue, the 4th's backward mask in the RGB layer's
    dgrad epilogue) against the same network
    with plain nn.ReLU modules, bf16 autocast, channels-last: output and every parameter
    and input gradient bit for bit (ReLU commutes with the bf16 rounding; the masks are the
    same comparisons).  MIOpen (the 200 -> 200 layers' backward) is pinned to deterministic
    solutions: its default weight-gradient kernels may accumulate in any order."""
    from lie_vae.experiments import nets
    monkeypatch.setattr(torch.backends.cudnn, "deterministic", True)
    monkeypatch.setattr(torch.backends.cudnn, "benchmark", False)
    torch.manual_seed(5)
    mods = []
    for fused in (True, False):
        monkeypatch.setattr(nets, "FUSED_RELU", fused)
        mods.append(nets.DeconvNet(1210, 200, rgb=True).to(gpu_device).to(memory_format=torch.channels_last))
    mods[1].load_state_dict(mods[0].state_dict())
    assert isinstance(mods[0][8], torch.nn.Identity) and mods[0][9].input_is_relu
    assert isinstance(mods[1][8], torch.nn.ReLU)
    z = torch.randn(6, 1210, device=gpu_device)
    gy = torch.randn(6, 3, 64, 64, device=gpu_device)
    outs = []
    for m in mods:
        zi = z.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = m(zi)
        (y.float() * gy).sum().backward()
        outs.append((y.detach(), zi.grad, [p.grad for p in m.parameters()]))
    assert torch.equal(outs[0][0], outs[1][0]), "forward"
    assert torch.equal(outs[0][1], outs[1][1]), "input gradient"
    for i, (a, b) in enumerate(zip(outs[0][2], outs[1][2])):
        assert torch.equal(a, b), f"parameter {i} gradient"


@pytest.mark.parametrize("N,C,H,W", [(64, 50, 32, 32), (16, 100, 16, 16), (32, 200, 8, 8), (64, 400, 4, 4),
                                     (3, 24, 5, 7), (2, 12, 3, 3), (2, 6, 4, 4)])
def test_fused_bn_leaky_relu_matches_float64(gpu_device, N, C, H, W):
    """FusedBatchNormLeakyReLU in training mode on a bf16 channels-last activation
    (lv_bn_lrelu_fwd_bf16 / lv_bn_lrelu_bwd_bf16, csrc/bn.hip; C = 6 takes the
    BatchNorm2d + leaky_relu fallback) against BatchNorm2d(training) + LeakyReLU(0.2)
    evaluated in float64 on the same bf16 input: y within bf16 rounding (2^-8 |ref| +
    1e-3 rms), running statistics to 1e-5, and the backward -- with the activation mask
    taken from the kernel's own y (sign(y) = sign(z)) -- gx within 2^-7 |ref| + 2e-3 rms,
    gamma / beta gradients (fp32) within 1e-4 relative + 1e-4 rms.  The fallback (PyTorch's
    bf16 BatchNorm output, then leaky_relu in bf16: two roundings) is checked 4x looser."""
    from lie_vae import _lib
    from lie_vae.experiments.nets import FusedBatchNormLeakyReLU
    loose = 1.0 if _lib.load().lv_bn_supported(N * H * W, C) else 4.0
    g = torch.Generator().manual_seed(N + C * 3 + H)
    x = (torch.randn(N, C, H, W, generator=g) * 1.5 + 0.7).to(torch.bfloat16)
    gy = torch.randn(N, C, H, W, generator=g).to(torch.bfloat16)
    m = FusedBatchNormLeakyReLU(C, 0.2).to(gpu_device)
    with torch.no_grad():
        m.weight.copy_(torch.rand(C, generator=g) + 0.5)
        m.bias.copy_(torch.randn(C, generator=g) * 0.3)
        m.running_mean.copy_(torch.randn(C, generator=g) * 0.1)
        m.running_var.copy_(torch.rand(C, generator=g) + 0.5)
    rm0, rv0 = m.running_mean.double().cpu(), m.running_var.double().cpu()
    w64, b64 = m.weight.detach().double().cpu(), m.bias.detach().double().cpu()
    xd = x.to(gpu_device).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    y = m(xd)
    y.backward(gy.to(gpu_device).contiguous(memory_format=torch.channels_last))
    assert y.dtype == torch.bfloat16 and int(m.num_batches_tracked) == 1
    x64, g64 = x.double(), gy.double()
    P = N * H * W
    mean = x64.mean((0, 2, 3))
    var = x64.var((0, 2, 3), unbiased=False)
    inv = 1.0 / torch.sqrt(var + m.eps)
    xhat = (x64 - mean.view(1, -1, 1, 1)) * inv.view(1, -1, 1, 1)
    z = xhat * w64.view(1, -1, 1, 1) + b64.view(1, -1, 1, 1)
    yref = torch.where(z > 0, z, 0.2 * z)
    yd = y.detach().double().cpu()
    rms = yref.square().mean().sqrt()
    bad = (yd - yref).abs() > loose * (2.0 ** -8 * yref.abs() + 1e-3 * rms)
    assert not bad.any(), f"y: {int(bad.sum())} off, max {(yd - yref).abs().max():.3e}"
    torch.testing.assert_close(m.running_mean.double().cpu(), 0.9 * rm0 + 0.1 * mean, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(m.running_var.double().cpu(), 0.9 * rv0 + 0.1 * var * P / (P - 1),
                               rtol=1e-5, atol=1e-6)
    gz = torch.where(yd > 0, g64, 0.2 * g64)
    if loose > 1:  # the fallback's leaky_relu backward runs in bf16
        gz = gz.to(torch.bfloat16).double()
    gb = gz.sum((0, 2, 3))
    gw = (gz * xhat).sum((0, 2, 3))
    gx = (w64 * inv).view(1, -1, 1, 1) * (gz - gb.view(1, -1, 1, 1) / P - xhat * gw.view(1, -1, 1, 1) / P)
    for name, got, ref, rel, absr in (("gx", xd.grad, gx, 2.0 ** -7, 2e-3), ("gw", m.weight.grad, gw, 1e-4, 1e-4),
                                      ("gb", m.bias.grad, gb, 1e-4, 1e-4)):
        gd = got.double().cpu()
        rms = ref.square().mean().sqrt()
        bad = (gd - ref).abs() > loose * (rel * ref.abs() + absr * rms)
        assert not bad.any(), f"{name}: {int(bad.sum())} of {bad.numel()} off, max {(gd - ref).abs().max():.3e}"


def test_accumulate_bf16_into_f32_bitwise(gpu_device):
    """lv_accumulate_bf16_f32 (the bf16 training step's master-gradient accumulation,
    nets.py _CachedCast) against torch's acc + g.float(): bit for bit, for every alignment
    of the two pointers (peeled head, 8 / 4 / 2-byte gradient reads), sizes with a ragged
    tail, and n = 0."""
    from lie_vae._lib import call, stream
    torch.manual_seed(3)
    cases = [(0, 0, 0), (1, 0, 0), (2, 0, 3), (7, 0, 0), (4096 * 9 + 3, 0, 0), (2_000_003, 0, 0)]
    cases += [(1001, og, oa) for og in range(4) for oa in range(4)]  # every alignment pair
    for n, off_g, off_a in cases:
        gb = torch.randn(n + off_g, device=gpu_device).to(torch.bfloat16)
        ab = torch.randn(n + off_a, device=gpu_device)
        g, a = gb[off_g:], ab[off_a:]
        ref = a + g.float()
        call("lv_accumulate_bf16_f32", g.data_ptr(), a.data_ptr(), n, stream())
        torch.cuda.synchronize(gpu_device)
        assert torch.equal(a, ref), (n, off_g, off_a)
