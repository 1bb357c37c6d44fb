"""torch.autograd.Functions over the C ABI.  Forward and backward both run the HIP
kernels of liblievae_hip.so on the caller's current stream; nothing here computes on
the CPU.  The per-sample maps follow the input dtype as the reference's do (fp64 in ->
the ``*_f64`` kernels, fp64 out; anything else -> fp32); the Wigner-D / group-action
path is fp32 (the reference's own J is fp32, ``lie_tools.py:10-14``) and the S2S2
Gram–Schmidt is fp64, as in the reference (``reparameterize.py:195-197``)."""
import torch

from . import _lib
from ._lib import call, ptr, stream

F32 = torch.float32


def _prep(t, dtype=F32):
    _lib.require_device(t)
    return t.contiguous() if t.dtype == dtype else t.to(dtype).contiguous()


def _empty(shape, like, dtype=F32):
    return torch.empty(shape, device=like.device, dtype=dtype)


F64 = torch.float64


def _map_dtype(*ts):
    """Compute dtype of a per-sample map: fp64 if any floating input is fp64 (torch's
    promotion for the reference's expressions), else fp32."""
    return F64 if any(t is not None and t.dtype == F64 for t in ts) else F32


def _k(name, dtype):
    return name + "_f64" if dtype == F64 else name


def _flat(t, last):
    """View (..., *last) as (n, *last); returns the batch shape too."""
    lead = t.shape[: t.dim() - len(last)]
    n = 1
    for d in lead:
        n *= d
    return t.reshape(n, *last), lead, n


# ------------------------------------------------------------- unary maps
class _Unary(torch.autograd.Function):
    """Generic per-sample map x (n, *IN) -> y (n, *OUT) with a VJP kernel; fp32 or fp64
    following the input."""

    @staticmethod
    def forward(ctx, x, spec):
        fwd, bwd, ishape, oshape = spec
        dt = _map_dtype(x) if fwd in _F64_MAPS else F32
        xf, lead, n = _flat(_prep(x, dt), ishape)
        y = _empty((n, *oshape), xf, dt)
        call(_k(fwd, dt), ptr(xf), ptr(y), n, stream())
        ctx.save_for_backward(xf)
        ctx.spec, ctx.lead, ctx.n, ctx.dt = spec, lead, n, dt
        return y.reshape(*lead, *oshape)

    @staticmethod
    def backward(ctx, gy):
        (xf,) = ctx.saved_tensors
        fwd, bwd, ishape, oshape = ctx.spec
        gyf = _prep(gy, ctx.dt).reshape(ctx.n, *oshape)
        gx = _empty((ctx.n, *ishape), xf, ctx.dt)
        call(_k(bwd, ctx.dt), ptr(xf), ptr(gyf), ptr(gx), ctx.n, stream())
        return gx.reshape(*ctx.lead, *ishape), None


SO3_EXP = ("lv_so3_exp_fwd", "lv_so3_exp_bwd", (3,), (3, 3))
QUAT_TO_MAT = ("lv_quat_to_mat_fwd", "lv_quat_to_mat_bwd", (4,), (3, 3))
MAT_TO_QUAT = ("lv_mat_to_quat_fwd", "lv_mat_to_quat_bwd", (3, 3), (4,))
QUAT_TO_EAZYZ = ("lv_quat_to_eazyz_fwd", "lv_quat_to_eazyz_bwd", (4,), (3,))
MAT_TO_EAZYZ = ("lv_mat_to_eazyz_fwd", "lv_mat_to_eazyz_bwd", (3, 3), (3,))
SOFTPLUS = ("lv_softplus_fwd", "lv_softplus_bwd", (), ())
# maps with fp64 twins
_F64_MAPS = {s[0] for s in (SO3_EXP, QUAT_TO_MAT, MAT_TO_QUAT, QUAT_TO_EAZYZ, MAT_TO_EAZYZ)}


def unary(x, spec):
    return _Unary.apply(x, spec)


# ----------------------------------------------------------- binary maps
class _S2S1(torch.autograd.Function):
    @staticmethod
    def forward(ctx, axis, cs):
        dt = _map_dtype(axis, cs)
        a, lead, n = _flat(_prep(axis, dt), (3,))
        c, _, _ = _flat(_prep(cs, dt), (2,))
        r = _empty((n, 3, 3), a, dt)
        call(_k("lv_s2s1_fwd", dt), ptr(a), ptr(c), ptr(r), n, stream())
        ctx.save_for_backward(a, c)
        ctx.lead, ctx.n, ctx.dt = lead, n, dt
        return r.reshape(*lead, 3, 3)

    @staticmethod
    def backward(ctx, g):
        a, c = ctx.saved_tensors
        gf = _prep(g, ctx.dt).reshape(ctx.n, 3, 3)
        ga, gc = _empty((ctx.n, 3), a, ctx.dt), _empty((ctx.n, 2), a, ctx.dt)
        call(_k("lv_s2s1_bwd", ctx.dt), ptr(a), ptr(c), ptr(gf), ptr(ga), ptr(gc), ctx.n,
             stream())
        return ga.reshape(*ctx.lead, 3), gc.reshape(*ctx.lead, 2)


class _S2S2(torch.autograd.Function):
    @staticmethod
    def forward(ctx, v1, v2):
        f64 = torch.float64
        a, lead, n = _flat(_prep(v1, f64), (3,))
        b, _, _ = _flat(_prep(v2, f64), (3,))
        r = _empty((n, 3, 3), a, f64)
        call("lv_s2s2_fwd_f64", ptr(a), ptr(b), ptr(r), n, stream())
        ctx.save_for_backward(a, b)
        ctx.lead, ctx.n = lead, n
        return r.reshape(*lead, 3, 3)

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        gf = _prep(g, torch.float64).reshape(ctx.n, 3, 3)
        g1, g2 = torch.empty_like(a), torch.empty_like(b)
        call("lv_s2s2_bwd_f64", ptr(a), ptr(b), ptr(gf), ptr(g1), ptr(g2), ctx.n, stream())
        return g1.reshape(*ctx.lead, 3), g2.reshape(*ctx.lead, 3)


class _SO3Sample(torch.autograd.Function):
    """z[s, b] = mu[b] @ exp(v[s, b]) — reparameterize.py:269-273."""

    @staticmethod
    def forward(ctx, mu, v):
        dt = _map_dtype(mu, v)
        mu = _prep(mu, dt)
        v = _prep(v, dt)
        ns, B = v.shape[0], v.shape[1]
        assert mu.shape == (B, 3, 3) and v.shape == (ns, B, 3)
        z = _empty((ns, B, 3, 3), v, dt)
        call(_k("lv_so3_sample_fwd", dt), ptr(mu), ptr(v), ptr(z), ns, B, stream())
        ctx.save_for_backward(mu, v)
        ctx.dt = dt
        return z

    @staticmethod
    def backward(ctx, gz):
        mu, v = ctx.saved_tensors
        ns, B = v.shape[0], v.shape[1]
        gz = _prep(gz, ctx.dt)
        gmu, gv = torch.empty_like(mu), torch.empty_like(v)
        call(_k("lv_so3_sample_bwd", ctx.dt), ptr(mu), ptr(v), ptr(gz), ptr(gmu), ptr(gv), ns,
             B, stream())
        return gmu, gv


class _N0Sample(torch.autograd.Function):
    """v[s, b] = eps[s, b] * sigma[b] — reparameterize.py:137-141 (eps given)."""

    @staticmethod
    def forward(ctx, sigma, eps):
        sigma = _prep(sigma)
        eps = _prep(eps)
        ns, B = eps.shape[0], eps.shape[1]
        v = torch.empty_like(eps)
        call("lv_n0_sample_fwd", ptr(sigma), ptr(eps), ptr(v), ns, B, stream())
        ctx.save_for_backward(eps)
        return v

    @staticmethod
    def backward(ctx, gv):
        (eps,) = ctx.saved_tensors
        ns, B = eps.shape[0], eps.shape[1]
        gs = _empty((B, 3), eps)
        call("lv_n0_sample_bwd", ptr(eps), ptr(_prep(gv)), ptr(gs), ns, B, stream())
        return gs, None


class _SO3LogPosterior(torch.autograd.Function):
    """log q(exp(v) | sigma), 2k+1 wrapped terms — reparameterize.py:233-263."""

    @staticmethod
    def forward(ctx, v, sigma, k):
        v = _prep(v)
        sigma = _prep(sigma)
        ns, B = v.shape[0], v.shape[1]
        out = _empty((ns, B), v)
        call("lv_so3_log_posterior_fwd", ptr(v), ptr(sigma), ptr(out), ns, B, k, stream())
        ctx.save_for_backward(v, sigma)
        ctx.k = k
        return out

    @staticmethod
    def backward(ctx, g):
        v, sigma = ctx.saved_tensors
        ns, B = v.shape[0], v.shape[1]
        gv, gs = torch.empty_like(v), torch.empty_like(sigma)
        call("lv_so3_log_posterior_bwd", ptr(v), ptr(sigma), ptr(_prep(g)), ptr(gv), ptr(gs),
             ns, B, ctx.k, stream())
        return gv, gs, None


# ------------------------------------------------------------ group action
_WS_BYTES = {}   # (n, L, C, shared F) -> lv_group_action_bwd_workspace
_WS_BUF = {}     # (device index, raw stream) -> cached uint8 workspace (eager calls only)


def _bwd_workspace(n, L, C, shared, device):
    """The backward's workspace: its size queried once per shape, the buffer reused per
    (device, stream) for eager calls (stream order serialises its users).  Under graph
    capture a fresh allocation from the graph's pool keeps replays independent of eager
    calls on other streams."""
    key = (n, L, C, shared)
    nb = _WS_BYTES.get(key)
    if nb is None:
        nb = _WS_BYTES[key] = int(_lib.load().lv_group_action_bwd_workspace(n, L, C, shared))
    st = _lib.stream_of(device)
    if torch.cuda.is_current_stream_capturing():
        return torch.empty(max(nb, 1), device=device, dtype=torch.uint8), nb, st
    bkey = (device.index, st)
    buf = _WS_BUF.get(bkey)
    if buf is None or buf.numel() < nb:
        buf = _WS_BUF[bkey] = torch.empty(max(nb, 1 << 20), device=device, dtype=torch.uint8)
    return buf, nb, st


class _GroupAction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, angles, spec, L, transpose, out_dtype):
        angles = _prep(angles)
        n = angles.shape[0]
        M = (L + 1) ** 2
        C = spec.shape[-1]
        stride = 0 if spec.dim() == 2 else M * C
        dt = _lib.LV_DTYPE_BF16 if out_dtype == torch.bfloat16 else _lib.LV_DTYPE_F32
        out = _empty((n, M, C), angles, out_dtype)
        call("lv_group_action_fwd", ptr(angles), ptr(spec), stride, ptr(out), dt, n, L, C,
             int(transpose), stream())
        ctx.save_for_backward(angles, spec)
        ctx.L, ctx.transpose, ctx.stride = L, transpose, stride
        return out

    @staticmethod
    def backward(ctx, gout):
        angles, spec = ctx.saved_tensors
        n, L, C = angles.shape[0], ctx.L, spec.shape[-1]
        gout = _prep(gout)
        gang = torch.empty_like(angles)
        gspec = torch.empty_like(spec)
        ws, ws_bytes, st = _bwd_workspace(n, L, C, int(ctx.stride == 0), angles.device)
        call("lv_group_action_bwd", ptr(angles), ptr(spec), ctx.stride, ptr(gout), ptr(gang),
             ptr(gspec), n, L, C, int(ctx.transpose), ws.data_ptr(), ws_bytes, st)
        return gang, gspec, None, None, None


def _check_spectrum(spectrum, n, L, what):
    """The shape contract of block_wigner_matrix_multiply (lie_tools.py:226-253), where
    the reference's bmm would raise: spectrum (M, C) or (n, M, C) with M = (L+1)^2.  A
    stride-0 batch expand of (M, C) (ActionNet's item_rep, decoders.py:53) collapses to
    the shared form.  Checked here because the kernels trust these sizes."""
    M = (L + 1) ** 2
    assert spectrum.dim() in (2, 3), f"{what}: spectrum must be (M,C) or (n,M,C), " \
                                     f"got {tuple(spectrum.shape)}"
    assert spectrum.shape[-2] == M, f"{what}: spectrum rows {spectrum.shape[-2]} != " \
                                    f"(L+1)^2 = {M}"
    if spectrum.dim() == 3:
        assert spectrum.shape[0] == n, f"{what}: spectrum batch {spectrum.shape[0]} != " \
                                       f"number of samples {n}"
        if spectrum.stride(0) == 0:
            # (M,C) passed once; autograd routes dF through expand back to item_rep
            spectrum = spectrum.as_strided(spectrum.shape[1:], spectrum.stride()[1:])
    return spectrum


def _check_out_dtype(out_dtype, what):
    """The kernels write fp32 or bf16 output only; anything else would be written with
    the wrong element size (checked before either path, Python or C++ operator)."""
    if out_dtype not in (torch.float32, torch.bfloat16):
        raise ValueError(f"{what}: out_dtype must be torch.float32 or torch.bfloat16, "
                         f"got {out_dtype}")


def group_action(angles, spectrum, L, transpose=False, out_dtype=F32):
    """block_wigner_matrix_multiply on the HIP path; angles (n,3), spectrum (M,C),
    (n,M,C) or a stride-0 expand of (M,C)."""
    assert angles.dim() == 2 and angles.shape[1] == 3, \
        f"angles must be (n,3), got {tuple(angles.shape)}"
    _check_out_dtype(out_dtype, "group_action")
    spectrum = _check_spectrum(spectrum, angles.shape[0], L, "group_action")
    _lib.require_device(angles, spectrum)
    return _GroupAction.apply(angles, _contig(spectrum), L, transpose, out_dtype)


def _contig(t):
    return t.contiguous() if t.dtype == F32 else t.float().contiguous()


def _f32c(t):
    """t itself when already fp32 and contiguous (the common case: no dispatcher call)."""
    return t if t.dtype == F32 and t.is_contiguous() else t.to(F32).contiguous()


class _FusedExpAction(torch.autograd.Function):
    """mu@exp(v) -> ZYZ -> block D·F in one launch; backward = one tile-kernel launch
    (group-action backward) + one launch of the dF slab reduce with the exp -> ZYZ VJP
    beside it.
    Host path kept short (the eager training direction is host-bound at config 2): no
    conversion calls on already-fp32 contiguous inputs, the workspace cached per stream."""

    @staticmethod
    def forward(ctx, mu, v, spec, L, transpose, out_dtype):
        v = _f32c(v)
        n = v.shape[0]
        mu_c = _f32c(mu) if mu is not None else None
        M = (L + 1) ** 2
        C = spec.shape[-1]
        dev = v.device
        out = torch.empty((n, M, C), device=dev, dtype=out_dtype)
        ang = torch.empty((n, 3), device=dev, dtype=F32)
        call("lv_fused_exp_action_fwd", None if mu_c is None else mu_c.data_ptr(), v.data_ptr(),
             spec.data_ptr(), 0, out.data_ptr(),
             _lib.LV_DTYPE_BF16 if out_dtype == torch.bfloat16 else _lib.LV_DTYPE_F32,
             ang.data_ptr(), n, L, C, int(transpose), _lib.stream_of(dev))
        ctx.save_for_backward(mu_c, v, spec, ang)
        ctx.L, ctx.transpose = L, transpose
        return out

    @staticmethod
    def backward(ctx, gout):
        mu, v, spec, ang = ctx.saved_tensors
        n, L, C = v.shape[0], ctx.L, spec.shape[-1]
        gout = _f32c(gout)
        dev = v.device
        gspec, gv = torch.empty_like(spec), torch.empty_like(v)
        gmu = torch.empty_like(mu) if mu is not None else None
        ws, ws_bytes, st = _bwd_workspace(n, L, C, 1, dev)
        call("lv_fused_exp_action_bwd", None if mu is None else mu.data_ptr(), v.data_ptr(),
             ang.data_ptr(), spec.data_ptr(), gout.data_ptr(),
             None if gmu is None else gmu.data_ptr(), gv.data_ptr(), gspec.data_ptr(), n, L, C,
             int(ctx.transpose), ws.data_ptr(), ws_bytes, st)
        return gmu, gv, gspec, None, None, None


_TORCH_OPS = _lib.load_torch_ops()  # liblievae_torch.so: the op as a C++ autograd function


def fused_exp_action(mu, v, spectrum, L, transpose=False, out_dtype=F32):
    """(mu (n,3,3) or None, v (n,3), spectrum (M,C) or a stride-0 expand of it) ->
    (n, M, C).  The fused kernel takes a shared spectrum only (ActionNet's item_rep);
    a per-sample spectrum goes through group_action.  Runs as the C++ operator
    torch.ops.lievae.fused_exp_action (csrc/torch_ops.cpp: forward, backward and autograd
    bookkeeping without Python frames) when liblievae_torch.so is built, else through the
    Python autograd.Function below -- the same kernels either way."""
    assert v.dim() == 2 and v.shape[1] == 3, f"v must be (n,3), got {tuple(v.shape)}"
    n = v.shape[0]
    if mu is not None:
        assert tuple(mu.shape) == (n, 3, 3), f"mu must be ({n},3,3), got {tuple(mu.shape)}"
    _check_out_dtype(out_dtype, "fused_exp_action")
    spectrum = _check_spectrum(spectrum, n, L, "fused_exp_action")
    if spectrum.dim() != 2:
        raise ValueError("fused_exp_action takes a shared (M,C) spectrum; use group_action "
                         "for a per-sample (n,M,C) spectrum")
    _lib.require_device(v, spectrum, mu)
    if _TORCH_OPS:
        return torch.ops.lievae.fused_exp_action(mu, v, spectrum, L, bool(transpose),
                                                 out_dtype == torch.bfloat16)
    return _FusedExpAction.apply(mu, v, _f32c(spectrum), L, transpose, out_dtype)


def wigner_blocks(angles, L):
    """Packed D_0..D_L for each angle triple (debug / parity), (n, sum (2l+1)^2)."""
    angles = _prep(angles)
    n = angles.shape[0]
    tot = (L + 1) * (2 * L + 1) * (2 * L + 3) // 3
    D = _empty((n, tot), angles)
    call("lv_wigner_d_fwd", ptr(angles), ptr(D), n, L, stream())
    return D


s2s1 = _S2S1.apply
s2s2 = _S2S2.apply
so3_sample = _SO3Sample.apply
n0_sample = _N0Sample.apply
so3_log_posterior = _SO3LogPosterior.apply
