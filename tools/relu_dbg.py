import sys, torch
sys.path[:0] = ["lie-vae_amd", "."]
from lie_vae.experiments import nets
dev = torch.device("cuda:0")
torch.manual_seed(5)
mods = []
for fused in (True, False):
    nets.FUSED_RELU = fused
    mods.append(nets.DeconvNet(1210, 200, rgb=True).to(dev).to(memory_format=torch.channels_last))
mods[1].load_state_dict(mods[0].state_dict())
z = torch.randn(6, 1210, device=dev)
acts = [[], []]
for k, m in enumerate(mods):
    for i, layer in enumerate(m):
        layer.register_forward_hook(lambda mod, inp, out, i=i, k=k: acts[k].append((i, out.detach().float().clone())))
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(z)
for (i, a), (j, b) in zip(acts[0], acts[1]):
    d = (a - b).abs()
    print(i, type(mods[0][i]).__name__, type(mods[1][j]).__name__, tuple(a.shape), "maxdiff", float(d.max()),
          "n", int((d > 0).sum()), "relu-equal", bool(torch.equal(a.clamp_min(0), b.clamp_min(0))))
# direct kernel check: layer 3 fused relu_out vs unfused + relu
x = acts[1][1][1].to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
from lie_vae.experiments.nets import _Deconv4s2
w = mods[0][3].weight.to(torch.bfloat16); b = mods[0][3].bias.float()
y0 = _Deconv4s2.apply(x, w, b, 0); y1 = _Deconv4s2.apply(x, w, b, 1)
print("relu_out kernel vs relu(plain):", bool(torch.equal(y1, torch.relu(y0))), float((y1.float() - torch.relu(y0).float()).abs().max()))
