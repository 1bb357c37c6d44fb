"""Host-side dispatch of the library's convolution layers (lie_vae/experiments/nets.py): which
inputs take the HIP kernels and which fall back to the plain torch layer.  CPU only (no
kernel launch): a CPU tensor never takes a kernel path, and the layers keep the reference
modules' parameters and state_dict keys (reference experiments/nets.py:33-75)."""
import torch

from lie_vae.experiments import nets


def test_fp32_layers_dispatch_conditions():
    m = nets.MfmaConvTranspose2d(200, 200, 4, 2, 1)
    x = torch.randn(2, 200, 4, 4)
    assert not m._mfma_f32_ok(x)                     # CPU tensor: plain layer
    ref = torch.nn.ConvTranspose2d(200, 200, 4, 2, 1)
    ref.load_state_dict(m.state_dict())
    torch.testing.assert_close(m(x), ref(x))
    assert set(m.state_dict()) == {"weight", "bias"}
    c = nets.MfmaDgradConv2d(200, 400, 4, 2, 1)
    xc = torch.randn(2, 200, 8, 8, requires_grad=True)
    assert not c._ok_f32(xc)
    refc = torch.nn.Conv2d(200, 400, 4, 2, 1)
    refc.load_state_dict(c.state_dict())
    torch.testing.assert_close(c(xc), refc(xc))


def test_deconvnet_twin_flags_follow_the_fp32_chain():
    """DeconvNet marks the two 200 -> 200 layers whose consumer is itself a 200 -> 200 layer
    (modules 3 and 5) to write the channels-last twin; the last hidden layer (7) feeds the
    RGB layer (Cout = 3, not an fp32-MFMA layer) and does not."""
    d = nets.DeconvNet(1210, 200, rgb=True)
    flags = {i: getattr(m, "cl_twin_out", None) for i, m in enumerate(d)}
    if nets.FUSED_RELU and nets.MFMA_DECONV:
        assert flags[3] and flags[5] and not flags[7]
    keys = set(d.state_dict())
    assert {"1.weight", "3.weight", "5.weight", "7.weight", "9.weight"} <= keys
