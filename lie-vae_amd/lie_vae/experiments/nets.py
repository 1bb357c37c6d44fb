"""Encoder / decoder stacks used around the SO(3) latent — drop-in for
``lie_vae.experiments.nets`` (reference lie_vae/experiments/nets.py:7-90).

These dense convolutions are MFMA work and run through PyTorch-ROCm (MIOpen /
hipBLASLt); they are callers of the hot path, not part of it.

Two layers of the stacks are plain GEMMs in disguise and run as one:
  * the decoder's first ConvTranspose2d(M·C, h, 4, 1, 0) sees a 1x1 input (nets.py:66):
    out[b, (o, i, j)] = x[b, :] · W[:, o, i, j] + bias[o], a [B x M·C]·[M·C x 16h] GEMM;
  * the encoder's head Conv2d(8h, out, 4, 1, 0) sees a 4x4 input (nets.py:54):
    out[b, o] = <x[b], W[o]> + bias[o], a [B x 128h]·[128h x out] GEMM.
``GemmConvTranspose2d`` / ``GemmConv2d`` keep the nn.ConvTranspose2d / nn.Conv2d
parameters (same state_dict) and compute those shapes with one addmm (hipBLASLt, on
MFMA; bf16 under autocast) instead of MIOpen's convolution solvers; any other input
shape takes the convolution.  ``GEMM_LAYERS = False`` before building a model restores
plain convolutions (A/B).
"""
import contextlib

import torch
from torch import nn
from torch.nn import functional as F

GEMM_LAYERS = True


def use_packaged_miopen_db():
    """Point MIOpen at the find-db shipped with the package (lie_vae/data/miopen: MIOpen's
    find results for the config-3 / config-4 convolutions on MI355X, gfx950 with 256 CUs,
    made by tools/gen_miopen_db.sh), copied to a private temp directory because MIOpen
    writes next to it.  Immediate mode (torch.backends.cudnn.benchmark = False) then runs
    the recorded winners instead of its fallback heuristics, which pick ConvDirectNaive
    kernels (30-300 ms per call) for several NHWC bf16 shapes.  Must run before the
    process's first convolution; a MIOPEN_USER_DB_PATH already set is left alone.  Returns
    the directory in use (None if the package has no db).  The private copy is removed at
    interpreter exit (atexit), so repeated runs and DP ranks leave nothing in the temp
    directory."""
    import atexit
    import os
    import shutil
    import tempfile
    if os.environ.get("MIOPEN_USER_DB_PATH"):
        return os.environ["MIOPEN_USER_DB_PATH"]
    src = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data", "miopen")
    if not os.path.isdir(src):
        return None
    dst = tempfile.mkdtemp(prefix="lievae_miopen_db_")
    atexit.register(shutil.rmtree, dst, True)
    for f in os.listdir(src):
        shutil.copy(os.path.join(src, f), dst)
    os.environ["MIOPEN_USER_DB_PATH"] = dst
    return dst


def _cl(t):
    return t.dim() == 4 and not t.is_contiguous() and t.is_contiguous(memory_format=torch.channels_last)


# ---- bf16 copies of the conv parameters, refreshed once per optimizer step
# Under bf16 autocast every conv / deconv casts its fp32 weight and bias to bf16 on every
# forward (one copy kernel per tensor: 24 per config-3 step).  Bf16ParamCache keeps bf16
# copies that DPTrainer refreshes with ONE multi-tensor copy after each optimizer step; a
# layer uses its copy only while it is current (same storage, same in-place version as at
# the refresh), else it casts as before.  The copy enters autograd through _CachedCast,
# whose backward is the cast's (gradient to fp32).
class _CachedCast(torch.autograd.Function):
    """Backward: the cast's (gradient to fp32) -- or, when the parameter's .grad is a
    gradient-bucket view of DPTrainer (``p._lv_grad_sink`` set by BucketedAllReduce), the
    bf16 gradient added into .grad in place by the library's one-pass kernel
    (lv_accumulate_bf16_f32; torch's mixed-dtype add_ runs a non-vectorised kernel, ~50 us
    per conv weight) and no gradient returned: one kernel per parameter instead of a cast
    and AccumulateGrad's add (22 + 22 tiny kernels per config-3 step).

    The bucket's accounting stays with the parameter's post-accumulate hook: autograd runs
    a leaf's AccumulateGrad once per backward, after every path into it (this node's None
    included), and fires the hook then -- so however many times the cached copy (or the
    parameter directly) entered the graph, every contribution is in the bucket before its
    hook counts the parameter, once.  (Round 4 also called the hook from here: with the
    hook's own call that counted a parameter twice and could launch a bucket's all-reduce
    early; BucketedAllReduce now refuses a second count in one step.)"""

    @staticmethod
    def forward(ctx, p, pb):
        ctx.dt = p.dtype
        ctx.p = p
        return pb.view_as(pb)

    @staticmethod
    def backward(ctx, g):
        p = ctx.p
        gr = p.grad
        if getattr(p, "_lv_grad_sink", None) is not None and gr is not None and not torch.is_grad_enabled():
            if (gr.is_cuda and g.dtype == torch.bfloat16 and gr.dtype == torch.float32 and g.shape == gr.shape
                    and g.stride() == gr.stride()
                    and (gr.is_contiguous() or (gr.dim() == 4 and gr.is_contiguous(memory_format=torch.channels_last)))):
                from .. import _lib
                _lib.call("lv_accumulate_bf16_f32", g.data_ptr(), gr.data_ptr(), gr.numel(),
                          _lib.stream_of(gr.device))
            else:
                gr.add_(g)
            return None, None
        return g.to(ctx.dt), None


def bf16_param(p):
    """p as bf16: the cached copy while it is current, else p.to(bfloat16)."""
    if p is None:
        return None
    e = getattr(p, "_lv_bf16", None)
    if e is not None and e[1] == p._version and e[2] == p.data_ptr():
        return _CachedCast.apply(p, e[0])
    return p.to(torch.bfloat16)


class Bf16ParamCache:
    """bf16 copies of the weights and biases of a model's convolution layers (the tensors
    autocast would cast per forward); refresh() after every optimizer step."""

    def __init__(self, model):
        self.src = [p for m in model.modules() if isinstance(m, (nn.Conv2d, nn.ConvTranspose2d))
                    for p in (m.weight, m.bias) if p is not None and p.dtype == torch.float32]
        self.dst = [torch.empty_like(p, dtype=torch.bfloat16) for p in self.src]
        self.refresh()

    @torch.no_grad()
    def refresh(self):
        if self.src:
            torch._foreach_copy_(self.dst, self.src)
        for p, d in zip(self.src, self.dst):
            p._lv_bf16 = (d, p._version, p.data_ptr())


def _autocast_bf16():
    return torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16


class GemmConvTranspose2d(nn.ConvTranspose2d):
    """ConvTranspose2d that runs a stride-1, unpadded layer on a 1x1 input as one GEMM."""

    def _gemm_shape(self, x):
        return (x.dim() == 4 and x.shape[-2:] == (1, 1) and self.stride == (1, 1)
                and self.padding == (0, 0) and self.output_padding == (0, 0)
                and self.dilation == (1, 1) and self.groups == 1)

    def forward(self, x, output_size=None):
        if output_size is not None or not self._gemm_shape(x):
            return super().forward(x, output_size)
        B, (k0, k1) = x.shape[0], self.kernel_size
        cl = _cl(self.weight)
        ac = _autocast_bf16()  # bf16 autocast: the cached bf16 parameters, explicit bf16 GEMM
        weight, bias = (bf16_param(self.weight), bf16_param(self.bias)) if ac else (self.weight, self.bias)
        # W (c_in, c_out, k0, k1) -> columns (o, i, j) [NCHW out] or (i, j, o) [NHWC out]
        w = (weight.permute(0, 2, 3, 1) if cl else weight).reshape(self.in_channels, -1)
        xm = x.reshape(B, self.in_channels)
        with torch.autocast("cuda", enabled=False) if ac else contextlib.nullcontext():
            if ac:
                xm = xm.to(torch.bfloat16)
            if bias is None:
                y = xm @ w
            else:
                b = bias.repeat(k0 * k1) if cl else bias.repeat_interleave(k0 * k1)
                y = torch.addmm(b, xm, w)
        if cl:
            return y.view(B, k0, k1, self.out_channels).permute(0, 3, 1, 2)
        return y.view(B, self.out_channels, k0, k1)


class GemmConv2d(nn.Conv2d):
    """Conv2d that runs a stride-1, unpadded layer whose input is exactly one kernel
    window (k x k -> 1x1) as one GEMM."""

    def _gemm_shape(self, x):
        return (x.dim() == 4 and tuple(x.shape[-2:]) == tuple(self.kernel_size)
                and self.stride == (1, 1) and self.padding == (0, 0)
                and self.dilation == (1, 1) and self.groups == 1
                and self.padding_mode == "zeros")

    def forward(self, x):
        if not self._gemm_shape(x):
            return super().forward(x)
        B = x.shape[0]
        ac = _autocast_bf16()
        weight, bias = (bf16_param(self.weight), bf16_param(self.bias)) if ac else (self.weight, self.bias)
        if _cl(x):  # NHWC memory: flatten (i, j, c) without a copy, reorder the weight
            xm = x.permute(0, 2, 3, 1).reshape(B, -1)
            w = weight.permute(0, 2, 3, 1).reshape(self.out_channels, -1)
        else:
            xm = x.reshape(B, -1)
            w = weight.reshape(self.out_channels, -1)
        with torch.autocast("cuda", enabled=False) if ac else contextlib.nullcontext():
            y = torch.nn.functional.linear(xm.to(torch.bfloat16) if ac else xm, w, bias)
        return y.view(B, self.out_channels, 1, 1)


# FUSED_BN_ACT: the encoder's BatchNorm2d + LeakyReLU pair as FusedBatchNormLeakyReLU (the
# library's deterministic bf16 channels-last kernels, csrc/bn.hip) + an Identity placeholder
# (same Sequential indices and state_dict keys).
FUSED_BN_ACT = True


class _BnLeakyReLU(torch.autograd.Function):
    """Training-mode BatchNorm2d + LeakyReLU on a channels-last bf16 activation through the
    library (lv_bn_lrelu_fwd_bf16 / lv_bn_lrelu_bwd_bf16, csrc/bn.hip): batch statistics,
    running-stat update, y = lrelu(gamma·xhat + beta) in one stats pass + one apply pass;
    backward = one reduce pass + one apply pass.  x is saved (not y): z is recomputed."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, momentum, eps, slope):
        from .. import _lib
        N, C, H, W = x.shape
        P = N * H * W
        dev = x.device
        y = torch.empty_like(x, memory_format=torch.channels_last)
        mean = torch.empty(C, device=dev, dtype=torch.float32)
        invstd = torch.empty(C, device=dev, dtype=torch.float32)
        ws = torch.empty(_lib.load().lv_bn_workspace_elems(P, C), device=dev, dtype=torch.float32)
        _lib.call("lv_bn_lrelu_fwd_bf16", x.data_ptr(), _lib.ptr(weight), _lib.ptr(bias),
                  _lib.ptr(running_mean), _lib.ptr(running_var), 1, momentum, eps, slope,
                  y.data_ptr(), mean.data_ptr(), invstd.data_ptr(), ws.data_ptr(), P, C, _lib.stream())
        ctx.save_for_backward(x, weight, bias, mean, invstd)
        ctx.slope = slope
        return y

    @staticmethod
    def backward(ctx, g):
        from .. import _lib
        x, weight, bias, mean, invstd = ctx.saved_tensors
        N, C, H, W = x.shape
        P = N * H * W
        g = g.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        gx = torch.empty_like(x, memory_format=torch.channels_last)
        gw = torch.empty_like(weight) if weight is not None else None
        gb = torch.empty_like(bias) if bias is not None else None
        ws = torch.empty(_lib.load().lv_bn_workspace_elems(P, C), device=x.device, dtype=torch.float32)
        _lib.call("lv_bn_lrelu_bwd_bf16", g.data_ptr(), x.data_ptr(), _lib.ptr(weight), _lib.ptr(bias),
                  mean.data_ptr(), invstd.data_ptr(), ctx.slope, gx.data_ptr(), _lib.ptr(gw), _lib.ptr(gb),
                  ws.data_ptr(), P, C, _lib.stream())
        return gx, gw, gb, None, None, None, None, None


class FusedBatchNormLeakyReLU(nn.BatchNorm2d):
    """BatchNorm2d(c) followed by LeakyReLU(slope) (the ConvNetBN pair, reference
    nets.py:33-57) in one module with BatchNorm2d's parameters, buffers and state_dict.
    Training-mode bf16 channels-last inputs on the GPU run the library's fused kernels;
    everything else (eval, fp32, NCHW, unsupported C) is BatchNorm2d + leaky_relu."""

    def __init__(self, num_features, negative_slope=0.2, **kw):
        super().__init__(num_features, **kw)
        self.negative_slope = negative_slope

    def _fused_ok(self, x):
        from .. import _lib
        if not (x.is_cuda and x.dim() == 4 and x.dtype == torch.bfloat16 and _cl(x)
                and self.training and self.track_running_stats and self.momentum is not None):
            return False
        # the kernels read gamma / beta / running stats as float* and write fp32 gamma /
        # beta gradients into buffers shaped like the parameters, and load x in 16-byte
        # pieces: a bf16 model (model.to(bfloat16)) or a misaligned view takes the fallback
        if x.data_ptr() % 16 or any(t is not None and (t.dtype != torch.float32 or not t.is_contiguous())
                                    for t in (self.weight, self.bias, self.running_mean, self.running_var)):
            return False
        N, C, H, W = x.shape
        return N * H * W > 1 and bool(_lib.load().lv_bn_supported(N * H * W, C))

    def forward(self, x):
        if not self._fused_ok(x):
            return F.leaky_relu(super().forward(x), self.negative_slope)
        self.num_batches_tracked.add_(1)
        return _BnLeakyReLU.apply(x, self.weight, self.bias, self.running_mean, self.running_var,
                                  float(self.momentum), float(self.eps), float(self.negative_slope))


class SyncBatchNormLeakyReLU(nn.SyncBatchNorm):
    """SyncBatchNorm (global-batch statistics) + LeakyReLU: what to_sync_batchnorm turns a
    FusedBatchNormLeakyReLU into for data-parallel training (same state_dict keys)."""

    def __init__(self, num_features, negative_slope=0.2, **kw):
        super().__init__(num_features, **kw)
        self.negative_slope = negative_slope

    def forward(self, x):
        return F.leaky_relu(super().forward(x), self.negative_slope)


def to_sync_batchnorm(module, process_group=None):
    """torch.nn.SyncBatchNorm.convert_sync_batchnorm that keeps the activation of the fused
    BatchNorm + LeakyReLU layers (FusedBatchNormLeakyReLU -> SyncBatchNormLeakyReLU)."""
    if isinstance(module, FusedBatchNormLeakyReLU):
        out = SyncBatchNormLeakyReLU(module.num_features, module.negative_slope, eps=module.eps,
                                     momentum=module.momentum, affine=module.affine,
                                     track_running_stats=module.track_running_stats,
                                     process_group=process_group)
        if module.affine:
            with torch.no_grad():
                out.weight = module.weight
                out.bias = module.bias
        out.running_mean = module.running_mean
        out.running_var = module.running_var
        out.num_batches_tracked = module.num_batches_tracked
        out.training = module.training
        return out
    if isinstance(module, nn.modules.batchnorm._BatchNorm) and not isinstance(module, nn.SyncBatchNorm):
        return nn.SyncBatchNorm.convert_sync_batchnorm(module, process_group)
    for name, child in module.named_children():
        module.add_module(name, to_sync_batchnorm(child, process_group))
    return module


# The stride-2 ConvTranspose2d forward on the library's MFMA kernels (lv_deconv4s2_fwd_bf16
# and, for the RGB output layer, lv_deconv4s2_small_fwd_bf16; csrc/deconv.hip) when it runs
# in bf16 (autocast) on channels-last inputs; fp32 / NCHW / unsupported shapes keep MIOpen.
# Config 3 bf16: 7.41 -> 6.29 ms/step (dec5 forward 989 -> 77 us, dec2-4 2x faster).
MFMA_DECONV = True
# DeconvNet's ReLUs fused into the neighbouring MFMA layers (MfmaConvTranspose2d.relu_out /
# input_is_relu): the forward clamps and the largest ReLU backward (after the 4th layer, folded
# into the RGB layer's dgrad epilogue) leave the step.
FUSED_RELU = True


def _channel_sum(g):
    """sum over (n, h, w) of a channels-last bf16 (N, C, H, W) gradient: the library's
    fixed-order per-channel sum (lv_channel_sum_bf16), fp32."""
    from .. import _lib
    C = g.shape[1]
    P = g.numel() // C
    out = torch.empty(C, device=g.device, dtype=torch.float32)
    ws = torch.empty(max(1, _lib.load().lv_channel_sum_workspace_elems(P, C)), device=g.device,
                     dtype=torch.float32)
    _lib.call("lv_channel_sum_bf16", g.data_ptr(), out.data_ptr(), ws.data_ptr(), P, C, _lib.stream())
    return out


class _Deconv4s2(torch.autograd.Function):
    """y = conv_transpose2d(x, w, b, stride 2, padding 1), k = 4: forward on the MFMA
    kernels (x, w bf16; b fp32 added before the bf16 rounding).  Backward: for Cout <= 4
    the library's quad-view dgrad / wgrad / bias kernels (lv_deconv4s2_small_bwd_bf16);
    otherwise aten.convolution_backward on the saved bf16 operands (what MIOpen computes
    for the plain layer) for gx, gw and the library's per-channel sum for gb.

    flags (include/lievae.h): LV_DECONV_RELU_OUT (Cout > 4) returns relu(y) from the
    forward epilogue, and the backward masks gy by y > 0 (ReLU's backward against its
    output) before the layer's own -- unless SKIP_MASK says the consumer of y already
    returns a masked gradient; LV_DECONV_MASK_GX (Cout <= 4) masks the dgrad output by
    x > 0, for an x that is a ReLU output (the ReLU's backward in the layer's epilogue).
    Both reproduce the unfused nn.ReLU + layer bit for bit."""

    SKIP_MASK = 1 << 8  # python-side flag, never passed to the library

    @staticmethod
    def forward(ctx, x, w, b, flags=0):
        from .. import _lib
        N, Cin, H, W = x.shape
        Cout = w.shape[1]
        wc = w.contiguous()
        small = Cout <= 4  # the RGB output layer: quad GEMM over the 3x3 neighbourhood
        ok = _lib.LV_DECONV_MASK_GX if small else (_lib.LV_DECONV_RELU_OUT | _Deconv4s2.SKIP_MASK)
        assert flags & ~ok == 0, f"flags {flags} not supported for Cout={Cout}"
        pre = "lv_deconv4s2_small_" if small else "lv_deconv4s2_"
        wt = torch.empty(getattr(_lib.load(), pre + "packed_weight_elems")(Cin), device=x.device,
                         dtype=torch.bfloat16)
        y = torch.empty((N, Cout, 2 * H, 2 * W), device=x.device, dtype=torch.bfloat16,
                        memory_format=torch.channels_last)
        st = _lib.stream()
        _lib.call(pre + "pack_weight_bf16", wc.data_ptr(), wt.data_ptr(), Cin, Cout, st)
        args = (x.data_ptr(), wt.data_ptr(), None if b is None else b.data_ptr(), y.data_ptr(),
                N, H, W, Cin, Cout)
        if small:
            _lib.call("lv_deconv4s2_small_fwd_bf16", *args, st)
        else:
            _lib.call("lv_deconv4s2_fwd_bf16_ex", *args, flags & _lib.LV_DECONV_RELU_OUT, st)
        relu_out = bool(flags & _lib.LV_DECONV_RELU_OUT) and not flags & _Deconv4s2.SKIP_MASK
        ctx.save_for_backward(x, wc, *((y,) if relu_out else ()))
        ctx.has_bias = b is not None
        ctx.flags = flags
        ctx.w_cl = _cl(w)  # the gradient comes back in the parameter's memory format
        return y

    @staticmethod
    def backward(ctx, gy):
        from .. import _lib
        x, w = ctx.saved_tensors[:2]
        N, Cin, H, W = x.shape
        Cout = w.shape[1]
        gy = gy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        if ctx.flags & _lib.LV_DECONV_RELU_OUT and not ctx.flags & _Deconv4s2.SKIP_MASK:
            gy = torch.ops.aten.threshold_backward(gy, ctx.saved_tensors[2], 0)
        need_x, need_w, need_b = ctx.needs_input_grad[:3]
        need_b = need_b and ctx.has_bias
        if Cout <= 4:
            lib, st = _lib.load(), _lib.stream()
            gx = wd = gw = gb = ws = None
            if need_x:
                wd = torch.empty(lib.lv_deconv4s2_small_dgrad_weight_elems(Cin), device=x.device,
                                 dtype=torch.bfloat16)
                _lib.call("lv_deconv4s2_small_pack_dgrad_weight_bf16", w.data_ptr(), wd.data_ptr(),
                          Cin, Cout, st)
                gx = torch.empty_like(x, memory_format=torch.channels_last)
            if need_w or need_b:
                gw = torch.empty_like(w)
                gb = torch.empty(Cout, device=x.device, dtype=torch.float32) if need_b else None
                ws = torch.empty(max(1, lib.lv_deconv4s2_small_bwd_workspace_elems(N, H, W, Cin, Cout)),
                                 device=x.device, dtype=torch.float32)
            _lib.call("lv_deconv4s2_small_bwd_bf16_ex", x.data_ptr(), gy.data_ptr(),
                      None if wd is None else wd.data_ptr(), None if gx is None else gx.data_ptr(),
                      None if gw is None else gw.data_ptr(), None if gb is None else gb.data_ptr(),
                      None if ws is None else ws.data_ptr(), N, H, W, Cin, Cout, ctx.flags, st)
            return gx, (_like(gw, ctx.w_cl) if need_w else None), gb, None
        gx, gw, _ = torch.ops.aten.convolution_backward(
            gy, x, w, None, [2, 2], [1, 1], [1, 1], True, [0, 0], 1, [need_x, need_w, False])
        return gx, _like(gw, ctx.w_cl), (_channel_sum(gy) if need_b else None), None


# fp32 (the reference's precision, no autocast): the k4 s2 p1 layers with 4 < Cout <= 208
# run their forward on lv_deconv4s2_fwd_f32 (fp32 MFMA) instead of MIOpen; their backward
# stays aten.convolution_backward (MIOpen), as for nn.ConvTranspose2d.
MFMA_DECONV_F32 = True


class _Deconv4s2F32(torch.autograd.Function):
    """y = conv_transpose2d(x, w, b, stride 2, padding 1), k = 4, fp32 NCHW in and out: the
    forward on lv_deconv4s2_fwd_f32 (x read channels-last: x_cl if given, else one
    transposing copy; with twin also y channels-last as the second, non-differentiable
    output, else an empty tensor there), with
    LV_DECONV_RELU_OUT returning relu(y) (the backward then masks gy by y > 0, unless
    SKIP_MASK: the consumer of y returns a masked gradient).  Backward: gx, gw, gb by
    aten.convolution_backward on the saved fp32 operands, what nn.ConvTranspose2d runs."""

    @staticmethod
    def forward(ctx, x, w, b, flags=0, x_cl=None, twin=False):
        from .. import _lib
        N, Cin, H, W = x.shape
        Cout = w.shape[1]
        wc = w.contiguous()
        st = _lib.stream()
        wt = torch.empty(_lib.load().lv_deconv4s2_packed_weight_elems_f32(Cin), device=x.device,
                         dtype=torch.float32)
        _lib.call("lv_deconv4s2_pack_weight_f32", wc.data_ptr(), wt.data_ptr(), Cin, Cout, st)
        xc = x_cl if x_cl is not None else x.contiguous(memory_format=torch.channels_last)
        y = torch.empty((N, Cout, 2 * H, 2 * W), device=x.device, dtype=torch.float32)
        ycl = (torch.empty((N, Cout, 2 * H, 2 * W), device=x.device, dtype=torch.float32,
                           memory_format=torch.channels_last) if twin else None)
        _lib.call("lv_deconv4s2_fwd_f32", xc.data_ptr(), wt.data_ptr(), None if b is None else b.data_ptr(),
                  y.data_ptr(), None if ycl is None else ycl.data_ptr(), N, H, W, Cin, Cout,
                  flags & _lib.LV_DECONV_RELU_OUT, st)
        relu_out = bool(flags & _lib.LV_DECONV_RELU_OUT) and not flags & _Deconv4s2.SKIP_MASK
        ctx.save_for_backward(x, wc, *((y,) if relu_out else ()))
        ctx.has_bias = b is not None
        ctx.relu_out = relu_out
        ctx.w_cl = _cl(w)
        if ycl is None:
            ycl = y.new_empty(0)
        ctx.mark_non_differentiable(ycl)
        return y, ycl

    @staticmethod
    def backward(ctx, gy, _gycl):
        x, w = ctx.saved_tensors[:2]
        Cout = w.shape[1]
        if ctx.relu_out:
            gy = torch.ops.aten.threshold_backward(gy, ctx.saved_tensors[2], 0)
        need_x, need_w, need_b = ctx.needs_input_grad[:3]
        need_b = need_b and ctx.has_bias
        gx, gw, gb = torch.ops.aten.convolution_backward(
            gy, x, w, [Cout] if need_b else None, [2, 2], [1, 1], [1, 1], True, [0, 0], 1,
            [need_x, need_w, need_b])
        return gx, _like(gw, ctx.w_cl), gb, None, None, None


def _like(g, channels_last):
    """A weight gradient in its parameter's memory format (a channels-last model keeps
    channels-last weights; ``channels_last`` is _cl of the parameter as the layer received
    it): AccumulateGrad then stores it as is, and the optimizer sees params and grads of
    one layout -- the condition for torch.optim's foreach / fused Adam paths (otherwise
    Adam falls back to one chain of kernels per tensor)."""
    if g is None:
        return g
    return g.contiguous(memory_format=torch.channels_last) if channels_last else g.contiguous()


class MfmaConvTranspose2d(nn.ConvTranspose2d):
    """nn.ConvTranspose2d (same parameters / state_dict) whose k4 s2 p1 forward runs on
    the MFMA kernel for bf16 channels-last inputs (autocast bf16, or bf16 tensors).

    relu_out (a plain attribute, not state): the layer computes relu(layer(x)) --
    DeconvNet moves its nn.ReLU modules into the neighbouring layers this way
    (FUSED_RELU); the MFMA path fuses it for Cout > 4 into the kernel's epilogue,
    everything else applies F.relu.
    input_is_relu: x is a ReLU output (relu(x) = x), so only the ReLU's backward mask
    remains, in the RGB layer's dgrad epilogue; grad_masked_downstream (on the layer that
    produced that x with relu_out): its consumer returns the masked gradient, so its own
    backward skips the mask.  Either way the consumer's fallback path applies F.relu,
    whose backward masks."""

    relu_out = False
    input_is_relu = False
    grad_masked_downstream = False
    # fp32 path: also write y channels-last for a consumer that is itself an fp32 MFMA layer
    # (DeconvNet sets it): that layer then reads it instead of transposing y
    cl_twin_out = False

    def extra_repr(self):
        fl = [n for n in ("relu_out", "input_is_relu", "grad_masked_downstream") if getattr(self, n)]
        return super().extra_repr() + "".join(f", {n}=True" for n in fl)

    def _mfma_ok(self, x):
        return (x.is_cuda and x.dim() == 4 and _cl(x) and self.kernel_size == (4, 4)
                and self.stride == (2, 2) and self.padding == (1, 1)
                and self.output_padding == (0, 0) and self.dilation == (1, 1)
                and self.groups == 1 and self.in_channels % 8 == 0
                and ((self.out_channels % 8 == 0 and self.out_channels <= 208)
                     # the small-Cout backward holds Cin + 1 (bias) channels in <= 16
                     # 16-wide tiles (lv_deconv4s2_small_bwd_bf16: kBwMaxCt)
                     or (self.out_channels <= 4 and self.in_channels <= 248))
                and x.shape[0] <= 65535)

    def _mfma_f32_ok(self, x):
        return (MFMA_DECONV_F32 and x.is_cuda and x.dim() == 4 and x.dtype == torch.float32
                and self.weight.dtype == torch.float32 and not torch.is_autocast_enabled("cuda")
                and self.kernel_size == (4, 4) and self.stride == (2, 2) and self.padding == (1, 1)
                and self.output_padding == (0, 0) and self.dilation == (1, 1) and self.groups == 1
                and self.in_channels % 4 == 0 and 4 < self.out_channels <= 208)

    def forward(self, x, output_size=None):
        F_ = torch.nn.functional
        if output_size is None and self._mfma_f32_ok(x):
            from .. import _lib
            flags = ((_lib.LV_DECONV_RELU_OUT if self.relu_out else 0)
                     | (_Deconv4s2.SKIP_MASK if self.relu_out and self.grad_masked_downstream else 0))
            tw = None if self.input_is_relu else getattr(x, "_lv_cl_twin", None)
            x_cl = tw[0] if tw is not None and tw[1] == x._version else None
            y, ycl = _Deconv4s2F32.apply(F_.relu(x) if self.input_is_relu else x, self.weight, self.bias,
                                         flags, x_cl, self.cl_twin_out)
            if self.cl_twin_out:
                y._lv_cl_twin = (ycl, y._version)
            return y
        bf16 = x.dtype == torch.bfloat16 or (
            torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16)
        if output_size is not None or not bf16 or not self._mfma_ok(x):
            y = super().forward(F_.relu(x) if self.input_is_relu else x, output_size)
            return F_.relu(y) if self.relu_out else y
        from .. import _lib
        small = self.out_channels <= 4
        flags = ((_lib.LV_DECONV_MASK_GX if self.input_is_relu and small else 0)
                 | (_lib.LV_DECONV_RELU_OUT if self.relu_out and not small else 0)
                 | (_Deconv4s2.SKIP_MASK if self.relu_out and self.grad_masked_downstream and not small else 0))
        with torch.autocast("cuda", enabled=False):
            xb = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
            if self.input_is_relu and not small:
                xb = F_.relu(xb)
            y = _Deconv4s2.apply(xb, bf16_param(self.weight),
                                 None if self.bias is None else self.bias.float(), flags)
            return F_.relu(y) if self.relu_out and small else y


# The encoder's strided Conv2d(c_in, c_out, 4, 2, 1) backward-data on the library's MFMA
# transposed-convolution kernel: gx = conv_transpose2d(gy, W, stride 2, padding 1) is exactly
# lv_deconv4s2_fwd_bf16 with the Conv2d weight (c_out, c_in, 4, 4) read as a
# ConvTranspose2d(c_out, c_in) weight.  MIOpen runs these dgrads at ~100-120 TFLOP/s
# (profiles/r03_train_config3_bf16_fused_steady_kernels.txt, igemm_bwd).  Forward and the
# weight / bias gradients stay on MIOpen.
MFMA_CONV_DGRAD = True


class _Conv4s2(torch.autograd.Function):
    """y = conv2d(x, w, b, stride 2, padding 1), k = 4, bf16 channels-last: forward and
    gw / gb by MIOpen (torch), gx by lv_deconv4s2_fwd_bf16 (fp32 accumulation, one bf16
    rounding)."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.has_bias = b is not None
        ctx.w_cl = _cl(w)
        return torch.nn.functional.conv2d(x, w, b, 2, 1)

    @staticmethod
    def backward(ctx, gy):
        from .. import _lib
        x, w = ctx.saved_tensors
        N, ci, H, W = x.shape
        co = w.shape[0]
        gy = gy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        need_x, need_w, need_b = ctx.needs_input_grad
        need_b = need_b and ctx.has_bias
        gx = gw = gb = None
        if need_x:
            st = _lib.stream()
            wt = torch.empty(_lib.load().lv_deconv4s2_packed_weight_elems(co), device=x.device,
                             dtype=torch.bfloat16)
            _lib.call("lv_deconv4s2_pack_weight_bf16", w.contiguous().data_ptr(), wt.data_ptr(), co, ci, st)
            gx = torch.empty_like(x, memory_format=torch.channels_last)
            _lib.call("lv_deconv4s2_fwd_bf16", gy.data_ptr(), wt.data_ptr(), None, gx.data_ptr(),
                      N, H // 2, W // 2, co, ci, st)
        if need_w or need_b:
            _, gw, gb = torch.ops.aten.convolution_backward(
                gy, x, w, [co] if need_b else None, [2, 2], [1, 1], [1, 1], False, [0, 0], 1,
                [False, need_w, need_b])
        return gx, _like(gw, ctx.w_cl), gb


class _Conv4s2F32(torch.autograd.Function):
    """y = conv2d(x, w, b, stride 2, padding 1), k = 4, fp32 NCHW: forward and gw / gb by
    MIOpen (torch), gx by lv_deconv4s2_fwd_f32 (fp32 MFMA; gy read channels-last) -- the
    encoder's widest layer, whose dgrad MIOpen runs at ~50 TFLOP/s in fp32
    (profiles/r06_conv_layers_f32.txt)."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.has_bias = b is not None
        return torch.nn.functional.conv2d(x, w, b, 2, 1)

    @staticmethod
    def backward(ctx, gy):
        from .. import _lib
        x, w = ctx.saved_tensors
        N, ci, H, W = x.shape
        co = w.shape[0]
        need_x, need_w, need_b = ctx.needs_input_grad
        need_b = need_b and ctx.has_bias
        gx = gw = gb = None
        if need_x:
            st = _lib.stream()
            wt = torch.empty(_lib.load().lv_deconv4s2_packed_weight_elems_f32(co), device=x.device,
                             dtype=torch.float32)
            _lib.call("lv_deconv4s2_pack_weight_f32", w.contiguous().data_ptr(), wt.data_ptr(), co, ci, st)
            gyc = gy.contiguous(memory_format=torch.channels_last)
            gx = torch.empty_like(x, memory_format=torch.contiguous_format)
            _lib.call("lv_deconv4s2_fwd_f32", gyc.data_ptr(), wt.data_ptr(), None, gx.data_ptr(), None,
                      N, H // 2, W // 2, co, ci, 0, st)
        if need_w or need_b:
            _, gw, gb = torch.ops.aten.convolution_backward(
                gy, x, w, [co] if need_b else None, [2, 2], [1, 1], [1, 1], False, [0, 0], 1,
                [False, need_w, need_b])
        return gx, gw, gb


class MfmaDgradConv2d(nn.Conv2d):
    """nn.Conv2d (same parameters / state_dict) whose k4 s2 p1 input gradient runs on the
    library's MFMA transposed-convolution kernel for bf16 channels-last inputs (autocast
    bf16, or bf16 tensors) with c_out % 8 == 0, c_in % 4 == 0, c_in <= 208 and even H, W;
    everything else is nn.Conv2d."""

    def _ok(self, x):
        return (x.is_cuda and x.dim() == 4 and _cl(x) and x.requires_grad
                and self.kernel_size == (4, 4) and self.stride == (2, 2) and self.padding == (1, 1)
                and self.dilation == (1, 1) and self.groups == 1 and self.padding_mode == "zeros"
                and self.out_channels % 8 == 0 and self.in_channels % 4 == 0
                and self.in_channels <= 208 and x.shape[2] % 2 == 0 and x.shape[3] % 2 == 0)

    def _ok_f32(self, x):
        # fp32: where the kernel's 208-channel tiles are mostly used (c_in > 104: the
        # 200 -> 400 layer; narrower outputs leave most of its MFMA tiles empty)
        return (MFMA_DECONV_F32 and x.is_cuda and x.dim() == 4 and x.dtype == torch.float32
                and self.weight.dtype == torch.float32 and x.requires_grad
                and not torch.is_autocast_enabled("cuda") and self.kernel_size == (4, 4)
                and self.stride == (2, 2) and self.padding == (1, 1) and self.dilation == (1, 1)
                and self.groups == 1 and self.padding_mode == "zeros" and self.out_channels % 4 == 0
                and 104 < self.in_channels <= 208 and x.shape[2] % 2 == 0 and x.shape[3] % 2 == 0)

    def forward(self, x):
        if self._ok_f32(x):
            return _Conv4s2F32.apply(x, self.weight, self.bias)
        ac = _autocast_bf16()
        bf16 = x.dtype == torch.bfloat16 or ac
        if not bf16 or not self._ok(x):
            if not ac or self.padding_mode != "zeros":
                return super().forward(x)
            with torch.autocast("cuda", enabled=False):  # autocast's conv, cached bf16 params
                return torch.nn.functional.conv2d(x.to(torch.bfloat16), bf16_param(self.weight),
                                                  bf16_param(self.bias), self.stride, self.padding,
                                                  self.dilation, self.groups)
        with torch.autocast("cuda", enabled=False):
            xb = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
            return _Conv4s2.apply(xb, bf16_param(self.weight), bf16_param(self.bias))


def _conv(*a):
    return (GemmConv2d if GEMM_LAYERS else nn.Conv2d)(*a)


def _convt(*a):
    return (GemmConvTranspose2d if GEMM_LAYERS else nn.ConvTranspose2d)(*a)


def _convt_s2(*a):
    return (MfmaConvTranspose2d if MFMA_DECONV else nn.ConvTranspose2d)(*a)


class View(nn.Module):
    def __init__(self, *shape):
        super().__init__()
        self.shape = shape

    def forward(self, x):
        return x.view(*self.shape)


class Flatten(nn.Module):
    def forward(self, x):
        return x.view(x.size(0), -1)


def _down_stack(in_dims, hidden, out_dims, batch_norm):
    """64x64 -> 4x4 by four stride-2 4x4 convs (widths h, 2h, 4h, 8h), then 4x4 -> 1x1."""
    layers, c = [], in_dims
    for i, width in enumerate([hidden, hidden * 2, hidden * 4, hidden * 8]):
        layers.append((MfmaDgradConv2d if MFMA_CONV_DGRAD else nn.Conv2d)(c, width, 4, 2, 1))
        if batch_norm and FUSED_BN_ACT:
            layers += [FusedBatchNormLeakyReLU(width, 0.2), nn.Identity()]
        else:
            if batch_norm:
                layers.append(nn.BatchNorm2d(width))
            layers.append(nn.LeakyReLU(0.2, inplace=True))
        c = width
    layers += [_conv(c, out_dims, 4, 1, 0), Flatten()]
    return layers


class ConvNet(nn.Sequential):
    """nets.py:7-31 (no batch norm)."""

    def __init__(self, out_dims, hidden_dims=50, rgb=False):
        super().__init__(*_down_stack(3 if rgb else 1, hidden_dims, out_dims, False))


class ConvNetBN(nn.Sequential):
    """nets.py:33-57 (batch norm after every strided conv)."""

    def __init__(self, out_dims, hidden_dims=50, rgb=False):
        super().__init__(*_down_stack(3 if rgb else 1, hidden_dims, out_dims, True))


class DeconvNet(nn.Sequential):
    """1x1 -> 64x64 transposed-conv stack — nets.py:60-75.  With FUSED_RELU (and the MFMA
    layers) the ReLUs after the 2nd, 3rd and 4th layers become those layers' relu_out
    (their forward epilogues apply them); the 4th's backward mask moves into the RGB
    layer's dgrad epilogue (input_is_relu / grad_masked_downstream), the other two masks
    stay in the layers' own backward.  The ReLU slots hold nn.Identity, so module indices
    and state_dict keys are the reference's."""

    def __init__(self, in_dims, hidden_dims, rgb=False):
        layers = [View(-1, in_dims, 1, 1), _convt(in_dims, hidden_dims, 4, 1, 0), nn.ReLU()]
        for _ in range(3):
            layers += [_convt_s2(hidden_dims, hidden_dims, 4, 2, 1), nn.ReLU()]
        layers.append(_convt_s2(hidden_dims, 3 if rgb else 1, 4, 2, 1))
        if FUSED_RELU and MFMA_DECONV:
            for i in (3, 5, 7):  # layers 2, 3, 4: relu_out
                layers[i].relu_out = True
                layers[i + 1] = nn.Identity()
            layers[7].grad_masked_downstream = True
            layers[9].input_is_relu = True
            layers[3].cl_twin_out = layers[5].cl_twin_out = True  # fp32: layers 3, 4 read them
        super().__init__(*layers)


class MLP(nn.Sequential):
    """nets.py:78-90."""

    def __init__(self, input_dims, output_dims, hidden_dims, num_layers=1, activation=nn.ReLU):
        if num_layers == 0:
            super().__init__(nn.Linear(input_dims, output_dims))
            return
        layers = [nn.Linear(input_dims, hidden_dims), activation()]
        for _ in range(num_layers - 1):
            layers += [nn.Linear(hidden_dims, hidden_dims), activation()]
        layers.append(nn.Linear(hidden_dims, output_dims))
        super().__init__(*layers)
