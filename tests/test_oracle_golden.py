"""Pin the CPU oracle (oracle/lie_ref.py) against golden vectors from the reference itself.

Fixtures come from oracle/gen_golden.py, which ran pimdh/lie-vae's own code (J injected).
The oracle restates the same op sequence on the same backend, so agreement is at the
level of fp32 rounding (most comparisons are bit-exact).
"""
import glob
import math
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, golden
from oracle import lie_ref as ref

T = torch.from_numpy


def close(a, b, rtol=1e-6, atol=1e-6):
    np.testing.assert_allclose(np.asarray(a), np.asarray(b), rtol=rtol, atol=atol)


def grad_of(fn, inputs, gout):
    xs = [T(np.array(x)).requires_grad_(True) for x in inputs]
    y = fn(*xs)
    (y * T(gout)).sum().backward()
    return y.detach().numpy(), [x.grad.numpy() for x in xs]


def test_conversions_forward_and_grad():
    g = golden("conversions.npz")
    for tag in ("", "_small", "_large"):
        y, (gv,) = grad_of(ref.so3_exp, [g[f"exp_v{tag}"]], g[f"exp_gR{tag}"])
        close(y, g[f"exp_R{tag}"])
        close(gv, g[f"exp_gv{tag}"], rtol=1e-5, atol=1e-5)
    assert np.isnan(ref.so3_exp(torch.zeros(1, 3)).numpy()).all()
    assert np.isnan(g["exp_zero"]).all()
    close(ref.mat_to_quat(T(g["haar_R"])), g["haar_q"])
    close(ref.mat_to_quat(T(g["gen_R"])), g["gen_q"])
    y, (gr,) = grad_of(ref.mat_to_eazyz, [g["haar_R"]], g["haar_gang"])
    close(y, g["haar_ang"])
    close(gr, g["haar_gR"], rtol=1e-5, atol=1e-5)
    _, (gr,) = grad_of(ref.mat_to_quat, [g["gen_R"]], g["haar_gq"])
    close(gr, g["gen_gR"], rtol=1e-5, atol=1e-5)
    y, (gq,) = grad_of(ref.quat_to_eazyz, [g["q_unit"]], g["haar_gang"])
    close(y, g["q_eazyz"])
    close(gq, g["q_geazyz"], rtol=1e-5, atol=1e-5)
    y, (gq,) = grad_of(ref.quat_to_mat, [g["q_in"]], g["q_gmat"])
    close(y, g["q_mat"])
    close(gq, g["q_gq"], rtol=1e-5, atol=1e-5)
    y, (ga, gc) = grad_of(ref.s2s1_exp, [g["s2s1_axis"], g["s2s1_cs"]], g["s2s1_gR"])
    close(y, g["s2s1_R"])
    close(ga, g["s2s1_gaxis"], rtol=1e-5, atol=1e-5)
    close(gc, g["s2s1_gcs"], rtol=1e-5, atol=1e-5)
    y, (g1, g2) = grad_of(ref.gram_schmidt_s2s2, [g["s2s2_v1"], g["s2s2_v2"]], g["s2s2_gR"])
    close(y, g["s2s2_R"], rtol=1e-12, atol=1e-12)
    close(g1, g["s2s2_gv1"], rtol=1e-10, atol=1e-10)
    close(g2, g["s2s2_gv2"], rtol=1e-10, atol=1e-10)
    close(ref.squash_to_eazyz(T(g["sq_v"])), g["sq_ang"])
    close(ref.mat_to_quat(T(g["edge_R"])), g["edge_q"])
    np.testing.assert_array_equal(ref.mat_to_eazyz(T(g["edge_R"])).numpy(), g["edge_ang"])


def test_wigner_blocks():
    g = golden("wigner.npz")
    for l in range(11):
        close(ref.wigner_d(T(g["ang"]), l), g[f"D{l}"], rtol=1e-5, atol=1e-6)
    close(ref.wigner_d(T(g["ang20"]), 20), g["D20"], rtol=1e-5, atol=1e-6)


def test_degree1_convention_pin():
    """D¹(R) = P Rᵀ Pᵀ with P: (x,y,z) -> (y,z,x)  (SURVEY.md Appendix A)."""
    g = golden("wigner.npz")
    r = T(g["prop_ra"]).double()
    d1 = ref.wigner_d(ref.mat_to_eazyz(r), 1)
    p = torch.tensor([[0., 1, 0], [0, 0, 1], [1, 0, 0]], dtype=torch.float64)
    close(d1, p @ r.transpose(1, 2) @ p.T, atol=2e-5, rtol=0)


@pytest.mark.parametrize("l", [0, 1, 2, 3, 5])
def test_reference_properties(l):
    """Orthogonality, inverse and D(b)D(a) = D(ab)  — lie_tools.py:337-357."""
    g = golden("wigner.npz")
    ra, rb = T(g["prop_ra"]), T(g["prop_rb"])
    wa = ref.wigner_d(ref.mat_to_eazyz(ra), l)
    wb = ref.wigner_d(ref.mat_to_eazyz(rb), l)
    wc = ref.wigner_d(ref.mat_to_eazyz(ra.bmm(rb)), l)
    eye = torch.eye(2 * l + 1).expand_as(wa)
    close(wa @ wa.transpose(-2, -1), eye, rtol=1e-4, atol=1e-5)
    winv = ref.wigner_d(ref.mat_to_eazyz(ra.transpose(1, 2).contiguous()), l)
    close(wa @ winv, eye, rtol=1e-4, atol=1e-5)
    close(wb.bmm(wa), wc, rtol=1e-3, atol=1e-3)


ACTION_FILES = sorted(glob.glob(os.path.join(GOLDEN, "action_*.npz")))


@pytest.mark.parametrize("path", ACTION_FILES, ids=[os.path.basename(p) for p in ACTION_FILES])
def test_action_forward_and_grad(path):
    name = os.path.basename(path)
    L, C, t, p = [int(x[1:]) for x in name[:-4].split("_")[1:]]
    g = golden(name)
    n = g["ang"].shape[0]

    def f(a, s):
        sx = s if p else s.expand(n, -1, -1)
        return ref.block_wigner_apply(a, sx, L, transpose=bool(t))

    y, (ga, gs) = grad_of(f, [g["ang"], g["spec"]], g["gout"])
    scale = np.abs(g["out"]).max()
    close(y, g["out"], rtol=1e-5, atol=1e-6 * scale)
    close(ga, g["gang"], rtol=1e-4, atol=1e-5 * np.abs(g["gang"]).max())
    close(gs, g["gspec"], rtol=1e-4, atol=1e-5 * np.abs(g["gspec"]).max())


def test_fused_exp_action():
    g = golden("fused_exp_action.npz")
    z = ref.so3_sample(T(g["mu"]), T(g["v"]))
    close(z, g["z"])
    ang = ref.mat_to_eazyz(z)
    close(ang, g["ang"])
    out = ref.action_decode(ang, T(g["item_rep"]), 10)
    close(out, g["out"], rtol=1e-5, atol=1e-5)


def test_log_posterior_and_kl():
    g = golden("reparam.npz")
    v = T(g["lp_v"]).requires_grad_(True)
    s = T(g["lp_sigma"]).requires_grad_(True)
    lp = ref.so3_log_posterior(v, s, k=10)
    close(lp.detach(), g["lp_out"], rtol=1e-6, atol=1e-5)
    (lp * T(g["lp_g"])).sum().backward()
    close(v.grad, g["lp_gv"], rtol=1e-4, atol=1e-4)
    close(s.grad, g["lp_gsigma"], rtol=1e-4, atol=1e-4)
    sig = ref.n0_sigma(T(g["n0_x"]))
    close(sig, g["n0_sigma"])
    close(ref.n0_kl(sig), g["n0_kl"])
    for mode in ("alg", "s2s2", "q", "s2s1"):
        v = T(g[f"{mode}_v"])
        close(ref.n0_sample(T(g[f"{mode}_sigma"]), T(g[f"{mode}_eps"])), v, rtol=0, atol=0)
        z = ref.so3_sample(T(g[f"{mode}_mu"]), v)
        close(z, g[f"{mode}_z"])
        lp = ref.so3_log_posterior(v, T(g[f"{mode}_sigma"]))
        close(lp, g[f"{mode}_logpost"], rtol=1e-6, atol=1e-5)
        kl = (lp - ref.so3_log_prior(z)).mean(0)
        close(kl, g[f"{mode}_kl"], rtol=1e-6, atol=1e-5)
    assert math.isclose(float(g["alg_logprior"].ravel()[0]), -math.log(8 * math.pi ** 2), rel_tol=1e-6)
