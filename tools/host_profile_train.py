"""cProfile of the eager config-3 bf16 training step's host side (DPTrainer.step, batch 512,
channels-last, autocast): where the ~3.5-4.4 ms of issue time per step goes.  Prints the
top functions by own time and by cumulative time over 20 profiled steps."""
import cProfile
import io
import pstats
import sys

import torch

sys.path[:0] = ["lie-vae_amd", "."]
from lie_vae.experiments import nets  # noqa: E402
from lie_vae.experiments.train_dp import DPTrainer  # noqa: E402
from lie_vae.experiments.vae import VAE  # noqa: E402

nets.use_packaged_miopen_db()
dev = torch.device("cuda:0")
torch.manual_seed(0)
model = VAE(latent_mode="so3", decoder_mode="action", degrees=10, rep_copies=10, rgb=True,
            batch_norm=True, deconv_hidden=200, mean_mode="s2s2").to(dev).to(memory_format=torch.channels_last)
tr = DPTrainer(model, lr=1e-3, clip_grads=1e-5, amp_dtype=torch.bfloat16, fused_adam=True)
x = torch.rand(512, 3, 64, 64, device=dev)
for _ in range(10):
    tr.step(x)
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(20):
    tr.step(x)
pr.disable()
torch.cuda.synchronize()
for key in ("tottime", "cumulative"):
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats(key).print_stats(35)
    print(s.getvalue())
