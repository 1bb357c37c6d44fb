"""ctypes binding of liblievae_hip.so (C ABI declared in include/lievae.h).

The library is built in-tree by ``make -C lie-vae_amd/csrc`` (or
``__graft_entry__.build()``).  There is no fallback: if the shared object is missing
or a call fails, this module raises.  Every entry point takes device pointers and the
caller's current HIP stream, so calls are asynchronous and graph-capturable.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LIEVAE_HIP_LIB", os.path.join(_HERE, "liblievae_hip.so"))

LV_DTYPE_F32 = 0
LV_DTYPE_BF16 = 1

_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_I = ctypes.c_int
_SZ = ctypes.c_size_t
_F = ctypes.c_float

# name -> argtypes (restype int unless noted)
_SIGS = {
    "lv_abi_version": [],
    "lv_max_degree": [],
    "lv_compute_units": [],
    "lv_so3_exp_fwd": [_P, _P, _I64, _P],
    "lv_so3_exp_bwd": [_P, _P, _P, _I64, _P],
    "lv_so3_sample_fwd": [_P, _P, _P, _I64, _I64, _P],
    "lv_so3_sample_bwd": [_P, _P, _P, _P, _P, _I64, _I64, _P],
    "lv_quat_to_mat_fwd": [_P, _P, _I64, _P],
    "lv_quat_to_mat_bwd": [_P, _P, _P, _I64, _P],
    "lv_mat_to_quat_fwd": [_P, _P, _I64, _P],
    "lv_mat_to_quat_bwd": [_P, _P, _P, _I64, _P],
    "lv_quat_to_eazyz_fwd": [_P, _P, _I64, _P],
    "lv_quat_to_eazyz_bwd": [_P, _P, _P, _I64, _P],
    "lv_mat_to_eazyz_fwd": [_P, _P, _I64, _P],
    "lv_mat_to_eazyz_bwd": [_P, _P, _P, _I64, _P],
    "lv_s2s1_fwd": [_P, _P, _P, _I64, _P],
    "lv_s2s1_bwd": [_P, _P, _P, _P, _P, _I64, _P],
    "lv_s2s2_fwd_f64": [_P, _P, _P, _I64, _P],
    "lv_s2s2_bwd_f64": [_P, _P, _P, _P, _P, _I64, _P],
    "lv_wigner_d_fwd": [_P, _P, _I64, _I, _P],
    "lv_action_fwd_plan": [_I, _I64, _I, _I64, _I, _I, _P],
    "lv_group_action_bwd_plan": [_I64, _I, _I, _I, _P],
    "lv_group_action_fwd": [_P, _P, _I64, _P, _I, _I64, _I, _I, _I, _P],
    "lv_group_action_bwd": [_P, _P, _I64, _P, _P, _P, _I64, _I, _I, _I, _P, _SZ, _P],
    "lv_exp_eazyz_vjp": [_P, _P, _P, _P, _P, _I64, _P],
    "lv_fused_exp_action_bwd": [_P, _P, _P, _P, _P, _P, _P, _P, _I64, _I, _I, _I, _P, _SZ, _P],
    "lv_fused_exp_action_fwd": [_P, _P, _P, _I64, _P, _I, _P, _I64, _I, _I, _I, _P],
    "lv_fused_exp_action_fwd_repeat": [_P, _P, _P, _I64, _P, _I, _P, _I64, _I, _I, _I, _I, _P],
    "lv_softplus_fwd": [_P, _P, _I64, _P],
    "lv_softplus_bwd": [_P, _P, _P, _I64, _P],
    "lv_n0_sample_fwd": [_P, _P, _P, _I64, _I64, _P],
    "lv_n0_sample_bwd": [_P, _P, _P, _I64, _I64, _P],
    "lv_so3_log_posterior_fwd": [_P, _P, _P, _I64, _I64, _I, _P],
    "lv_so3_log_posterior_bwd": [_P, _P, _P, _P, _P, _I64, _I64, _I, _P],
}
# fp64 twins of the per-sample maps (same argument lists, double pointers)
for _name in ("lv_so3_exp_fwd", "lv_so3_exp_bwd", "lv_so3_sample_fwd", "lv_so3_sample_bwd",
              "lv_exp_eazyz_vjp", "lv_quat_to_mat_fwd", "lv_quat_to_mat_bwd",
              "lv_mat_to_quat_fwd", "lv_mat_to_quat_bwd", "lv_quat_to_eazyz_fwd",
              "lv_quat_to_eazyz_bwd", "lv_mat_to_eazyz_fwd", "lv_mat_to_eazyz_bwd",
              "lv_s2s1_fwd", "lv_s2s1_bwd"):
    _SIGS[_name + "_f64"] = _SIGS[_name]
_SIGS["lv_deconv4s2_pack_weight_bf16"] = [_P, _P, _I, _I, _P]
_SIGS["lv_deconv4s2_fwd_bf16"] = [_P, _P, _P, _P, _I64, _I, _I, _I, _I, _P]
_SIGS["lv_deconv4s2_small_pack_weight_bf16"] = [_P, _P, _I, _I, _P]
_SIGS["lv_deconv4s2_small_fwd_bf16"] = [_P, _P, _P, _P, _I64, _I, _I, _I, _I, _P]
_SIGS["lv_deconv4s2_small_pack_dgrad_weight_bf16"] = [_P, _P, _I, _I, _P]
_SIGS["lv_deconv4s2_small_bwd_bf16"] = [_P, _P, _P, _P, _P, _P, _P, _I64, _I, _I, _I, _I, _P]
_SIGS["lv_deconv4s2_fwd_bf16_ex"] = [_P, _P, _P, _P, _I64, _I, _I, _I, _I, _I, _P]
_SIGS["lv_deconv4s2_small_bwd_bf16_ex"] = [_P, _P, _P, _P, _P, _P, _P, _I64, _I, _I, _I, _I, _I, _P]
LV_DECONV_RELU_OUT, LV_DECONV_MASK_GX = 1, 4  # include/lievae.h
_SIGS["lv_deconv4s2_pack_weight_f32"] = [_P, _P, _I, _I, _P]
_SIGS["lv_deconv4s2_fwd_f32"] = [_P, _P, _P, _P, _P, _I64, _I, _I, _I, _I, _I, _P]
_SIGS["lv_channel_sum_bf16"] = [_P, _P, _P, _I64, _I, _P]
_SIGS["lv_accumulate_bf16_f32"] = [_P, _P, _I64, _P]
_SIGS["lv_bn_lrelu_fwd_bf16"] = [_P, _P, _P, _P, _P, _I, _F, _F, _F, _P, _P, _P, _P, _I64, _I, _P]
_SIGS["lv_bn_lrelu_bwd_bf16"] = [_P, _P, _P, _P, _P, _P, _F, _P, _P, _P, _P, _I64, _I, _P]
_RESTYPES = {"lv_group_action_bwd_workspace": _SZ, "lv_last_error": ctypes.c_char_p,
             "lv_deconv4s2_packed_weight_elems": _SZ, "lv_deconv4s2_small_packed_weight_elems": _SZ,
             "lv_deconv4s2_packed_weight_elems_f32": _SZ,
             "lv_deconv4s2_small_dgrad_weight_elems": _SZ, "lv_deconv4s2_small_bwd_workspace_elems": _SZ,
             "lv_channel_sum_workspace_elems": _SZ, "lv_bn_workspace_elems": _SZ}
_SIGS_EXTRA = {"lv_group_action_bwd_workspace": [_I64, _I, _I, _I], "lv_last_error": [],
               "lv_deconv4s2_packed_weight_elems": [_I], "lv_deconv4s2_small_packed_weight_elems": [_I],
               "lv_deconv4s2_packed_weight_elems_f32": [_I],
               "lv_deconv4s2_small_dgrad_weight_elems": [_I],
               "lv_deconv4s2_small_bwd_workspace_elems": [_I64, _I, _I, _I, _I],
               "lv_channel_sum_workspace_elems": [_I64, _I],
               "lv_bn_supported": [_I64, _I], "lv_bn_workspace_elems": [_I64, _I]}

EXPORTED = sorted(list(_SIGS) + list(_SIGS_EXTRA))
# entry points of the A/B build only (liblievae_hip_ab.so, -DLV_AB_KNOBS; tools/ sweeps):
# bound when the loaded library has them, never part of the product header
_SIGS_AB = {"lv_deconv4s2_fwd_bf16_tile": [_P, _P, _P, _P, _I64, _I, _I, _I, _I, _I, _P]}

_lib = None


class LieVaeHipError(RuntimeError):
    pass


def load():
    """Load (once) and return the shared library; raise if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"lie_vae: HIP library not found at {LIB_PATH}; build it with "
            "`make -C lie-vae_amd/csrc` (or __graft_entry__.build()). There is no CPU fallback.")
    lib = ctypes.CDLL(LIB_PATH)
    for name, args in {**_SIGS, **_SIGS_EXTRA}.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = _RESTYPES.get(name, ctypes.c_int)
    for name, args in _SIGS_AB.items():
        if hasattr(lib, name):
            getattr(lib, name).argtypes = args
    _lib = lib
    return lib


def last_error():
    return load().lv_last_error().decode(errors="replace")


_fns = {}


def call(name, *args):
    """Invoke an entry point; non-zero return -> LieVaeHipError with the library message.
    (Bound functions are looked up once; pointers and the stream travel as plain ints.)"""
    fn = _fns.get(name)
    if fn is None:
        fn = _fns[name] = getattr(load(), name)
    rc = fn(*args)
    if rc != 0:
        raise LieVaeHipError(f"{name} failed ({rc}): {last_error()}")


PLAN_LEN = 40  # LV_PLAN_LEN
PLAN_FIELDS = ("tile", "blocks", "segments", "threads", "lds_bytes", "samples_per_group", "aux")


def plan(kind, *args):
    """Host-only launch plan ("fwd": fused, F_batch_stride, out_dtype, n, L, C;
    "bwd": n, L, C, shared_F) as a dict; no GPU call (include/lievae.h LV_PLAN_LEN)."""
    buf = (ctypes.c_int64 * PLAN_LEN)()
    call("lv_action_fwd_plan" if kind == "fwd" else "lv_group_action_bwd_plan", *args, buf)
    d = dict(zip(PLAN_FIELDS, buf[:7]))
    d["seg_lo"] = [x for x in buf[7:24] if x >= 0]
    d["seg_mask"] = list(buf[24:24 + d["segments"]])
    return d


TORCH_OPS_PATH = os.environ.get("LIEVAE_TORCH_OPS_LIB", os.path.join(_HERE, "liblievae_torch.so"))
_torch_ops = None


def load_torch_ops():
    """Register the C++ operators of liblievae_torch.so (csrc/torch_ops.cpp) with torch
    once; False when that library is not built (the Python autograd path is used then)."""
    global _torch_ops
    if _torch_ops is None:
        _torch_ops = False
        if os.path.exists(TORCH_OPS_PATH):
            load()  # the kernels' library first (the operators link against it)
            try:
                torch.ops.load_library(TORCH_OPS_PATH)
                _torch_ops = True
            except (OSError, RuntimeError) as e:  # stale build / torch ABI changed
                import warnings
                warnings.warn(f"lie_vae: {TORCH_OPS_PATH} did not load ({e}); the fused op "
                              "runs through the Python autograd path (same kernels). Rebuild "
                              "with `make -C lie-vae_amd/csrc`.")
    return _torch_ops


def stream():
    """The caller's current HIP stream (raw handle, as an int)."""
    return torch._C._cuda_getCurrentRawStream(torch.cuda.current_device())


def stream_of(device):
    """The current HIP stream of a tensor's device (raw handle, as an int)."""
    return torch._C._cuda_getCurrentRawStream(device.index)


def ptr(t):
    return t.data_ptr() if t is not None else None


def require_device(*tensors):
    """The HIP path only: refuse CPU tensors loudly instead of silently falling back, and
    tensors spread over several GPUs (the kernels take raw pointers of one device)."""
    dev = None
    for t in tensors:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError(
                "lie_vae ops run only on the MI355X HIP path (got a CPU tensor); "
                "move inputs to a cuda:N (HIP) device. There is no CPU fallback.")
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise RuntimeError(f"lie_vae ops need all inputs on one device (got {dev} and "
                               f"{t.device})")
