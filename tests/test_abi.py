"""CPU checks of the drop-in boundary: the C-ABI library loads without a GPU and exports
every entry point include/lievae.h declares; the Python API mirrors the reference names
and refuses CPU tensors (no silent fallback)."""
import os
import re

import pytest
import torch

from conftest import REPO


def header_symbols():
    text = open(os.path.join(REPO, "include", "lievae.h")).read()
    return sorted(set(re.findall(r"\b(lv_\w+)\s*\(", text)))


def test_library_exports_all_header_symbols():
    from lie_vae import _lib
    lib = _lib.load()
    syms = header_symbols()
    assert len(syms) >= 30
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(_lib.EXPORTED), set(syms) ^ set(_lib.EXPORTED)
    assert lib.lv_abi_version() == 1
    assert lib.lv_max_degree() == 20


def test_library_is_gfx950():
    from lie_vae import _lib
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_api_surface_matches_reference_names():
    import lie_vae.decoders as d
    import lie_vae.lie_tools as lt
    import lie_vae.reparameterize as rp
    import lie_vae.utils as u
    for name in ["j_matrix", "map_to_lie_algebra", "map_to_lie_vector", "rodrigues",
                 "s2s1rodrigues", "s2s2_gram_schmidt", "vector_to_eazyz", "log_map",
                 "group_matrix_to_quaternions", "quaternions_to_eazyz", "group_matrix_to_eazyz",
                 "quaternions_to_group_matrix", "wigner_d_matrix",
                 "block_wigner_matrix_multiply", "random_quaternions", "random_group_matrices"]:
        assert callable(getattr(lt, name)), name
    for name in ["Nreparameterize", "N0reparameterize", "SO3reparameterize", "AlgebraMean",
                 "QuaternionMean", "S2S1Mean", "S2S2Mean"]:
        assert isinstance(getattr(rp, name), type), name
    assert callable(d.ActionNet) and callable(d.MLPNet) and callable(u.logsumexp)


def test_cpu_tensors_fail_loudly():
    import lie_vae.lie_tools as lt
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        lt.rodrigues(torch.randn(4, 3))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        lt.block_wigner_matrix_multiply(torch.randn(4, 3), torch.randn(4, 16, 2), 3)


def test_shape_asserts_like_reference():
    import lie_vae.lie_tools as lt
    with pytest.raises(AssertionError):
        lt.group_matrix_to_quaternions(torch.randn(4, 3, 2))
    with pytest.raises(AssertionError):
        lt.quaternions_to_eazyz(torch.randn(4, 3))
    with pytest.raises(AssertionError):
        lt.wigner_d_matrix(torch.randn(4, 2), 1)


def test_hat_vee_roundtrip_cpu():
    """Pure data rearrangement (lie_tools.py:17-53) runs on any device."""
    import lie_vae.lie_tools as lt
    from oracle import lie_ref
    v = torch.randn(100, 3, dtype=torch.float64)
    m = lt.map_to_lie_algebra(v)
    assert torch.equal(m, lie_ref.hat(v))
    assert torch.equal(lt.map_to_lie_vector(m), v)


def test_j_table_matches_header_and_oracle():
    import numpy as np
    from lie_vae._jtab import j_numpy
    from oracle import lie_ref
    for l in (0, 1, 5, 10, 20):
        j = j_numpy(l)
        n = 2 * l + 1
        np.testing.assert_allclose(j @ j, np.eye(n), atol=1e-10)
        np.testing.assert_allclose(j, j.T, atol=0)
        np.testing.assert_array_equal(lie_ref.j_table(l).numpy(), j.astype(np.float32))
    hdr = open(os.path.join(REPO, "lie-vae_amd", "csrc", "j_tables.h")).read()
    assert "#define LV_J_LMAX 20" in hdr


def test_toy_dataset_host_side(tmp_path):
    """ToyDataset (datasets.py:129-162): seeded spectrum of norm 10, the generator refuses
    CPU tensors (the action runs only on the HIP path), and save/load round-trips through
    a weights_only torch.load."""
    from lie_vae.experiments.datasets import ToyDataset, toy_harmonics
    torch.manual_seed(0)
    h = toy_harmonics(6, 10)
    assert h.shape == (49, 10)
    assert torch.allclose(h.norm(), torch.tensor(10.0))
    torch.manual_seed(0)  # the caller seeds (datasets.py:144-145); same seed, same draw
    assert torch.equal(h, toy_harmonics(6, 10))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        ToyDataset.generate(n=8, degrees=6, device="cpu")
    q = torch.randn(5, 4)
    x = torch.randn(5, 49, 10)
    ds = ToyDataset(tensors=(q, h.expand(5, -1, -1), x))
    p = str(tmp_path / "toy.pt")
    ds.save(p)
    back = ToyDataset(path=p)
    assert len(back) == 5
    for a, b in zip(ds.tensors, back.tensors):
        assert torch.equal(a, b)


def test_spectrum_shape_contract_raises():
    """A spectrum whose batch, rows or rank disagree with the angles must raise before any
    kernel runs (the reference's bmm raises there; the kernels trust these sizes)."""
    import lie_vae._ops as ops
    import lie_vae.lie_tools as lt
    ang = torch.randn(6, 3)
    with pytest.raises(AssertionError, match="batch"):
        lt.block_wigner_matrix_multiply(ang, torch.randn(4, 16, 2), 3)
    with pytest.raises(AssertionError, match="rows"):
        lt.block_wigner_matrix_multiply(ang, torch.randn(6, 15, 2), 3)
    with pytest.raises(AssertionError, match="angles"):
        ops.group_action(torch.randn(6, 4), torch.randn(16, 2), 3)
    with pytest.raises(AssertionError, match="mu"):
        ops.fused_exp_action(torch.randn(5, 3, 3), torch.randn(6, 3), torch.randn(16, 2), 3)
    with pytest.raises(ValueError, match="shared"):
        ops.fused_exp_action(None, torch.randn(6, 3), torch.randn(6, 16, 2), 3)
    # a stride-0 expand of (M, C) is the shared form (and then hits the device check)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        ops.fused_exp_action(None, torch.randn(6, 3), torch.randn(16, 2).expand(6, -1, -1), 3)


def test_out_dtype_validated_before_any_path():
    """an out_dtype other than fp32 / bf16 would be written with the wrong
    element size by the kernels; both the Python and the C++ operator paths refuse it
    up front (ValueError, before the device check)."""
    from lie_vae import _ops
    v = torch.randn(4, 3)
    F = torch.randn(16, 2)
    for dt in (torch.float16, torch.float64, torch.int32):
        with pytest.raises(ValueError, match="out_dtype"):
            _ops.fused_exp_action(None, v, F, 3, out_dtype=dt)
        with pytest.raises(ValueError, match="out_dtype"):
            _ops.group_action(torch.randn(4, 3), F, 3, out_dtype=dt)


def test_require_device_refuses_cpu():
    """The CPU case (no device here); the mixed-device case is a GPU test
    (test_gpu_parity.py::test_torch_operator_refuses_cpu_or_mixed_inputs)."""
    from lie_vae import _lib
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        _lib.require_device(None, torch.randn(2))


def test_deconv_f32_argument_checks_before_any_launch():
    """lv_deconv4s2_pack_weight_f32 / lv_deconv4s2_fwd_f32 refuse shapes outside the fp32
    kernel's contract (Cin % 4 == 0, 1 <= Cout <= 208, a channels-last twin only with
    Cout % 4 == 0) with LV_ERR_ARG and a message, before touching the device; an empty
    batch is a no-op (LV_OK)."""
    import ctypes
    from lie_vae import _lib
    lib = _lib.load()
    P = ctypes.c_void_p(16)  # never dereferenced: the checks run first
    fwd = lib.lv_deconv4s2_fwd_f32
    assert lib.lv_deconv4s2_packed_weight_elems_f32(200) == 4 * 208 * 4 * 200 + 16
    assert lib.lv_deconv4s2_pack_weight_f32(P, P, 6, 200, None) == -1
    assert b"multiple of 4" in lib.lv_last_error()
    assert lib.lv_deconv4s2_pack_weight_f32(P, P, 200, 209, None) == -1
    assert fwd(P, P, None, P, None, 2, 4, 4, 6, 200, 0, None) == -1
    assert fwd(P, P, None, P, None, 2, 4, 4, 200, 209, 0, None) == -1
    assert fwd(P, P, None, P, P, 2, 4, 4, 200, 6, 0, None) == -1  # twin needs Cout % 4 == 0
    assert b"twin" in lib.lv_last_error()
    assert fwd(P, P, None, P, None, 2, 4, 4, 200, 200, 2, None) == -1  # unknown flag
    assert fwd(P, P, None, P, None, 0, 4, 4, 200, 200, 0, None) == 0   # empty batch
