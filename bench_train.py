#!/usr/bin/env python3
"""Training-step benchmark for BASELINE configs 3 and 4 (not the driver's bench.py).

Config 3: the full sphere-cube VAE (ConvNetBN encoder -> SO(3) reparam with S2S2 mean
-> action decoder l=10, C=10 -> DeconvNet(hidden 200), RGB 64x64), batch 512, one GPU.
Config 4: the same model, global batch 4096 data-parallel over N GPUs (512 per rank),
RCCL all-reduce of the gradients (lie_vae.experiments.train_dp).

One step = elbo forward (n=1) + backward + global-norm clip (1e-5) + Adam (lr 1e-3) —
the reference step of unsupervised.py:69-117 without its per-step host syncs.  Inputs:
synthetic x ~ U[0,1)^(B x 3 x 64 x 64) resident in HBM (the sphere-cube renders are not
available offline), seeded per rank.

  python bench_train.py                                   # config 3
  python bench_train.py --gpus 8 --global-batch 4096      # config 4 (spawns 8 ranks)
  python bench_train.py --gpus 2 --dry-run                # rank plumbing on CPU (gloo)
  python bench_train.py --iwae 64                         # IWAE LL eval, n=500 (f3)

``--iwae K`` times the reference's evaluation instead (main.py:134-139): the importance-
weighted log-likelihood with n = 500 samples over K test images, once one image per call
as the reference's batch-1 loader does, once ``--iwae-batch`` images per call; images
are sharded over ranks.

``--gpus N`` without a torch.distributed environment hands the script to
torch.distributed.run before any HIP call (lie_vae/experiments/launch.py).
"""
import argparse
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "lie-vae_amd"))
from lie_vae.experiments import launch  # noqa: E402  (no HIP call at import)

F32_PEAK_TFLOPS = 157.3  # MI355X f32 MFMA = f32 VALU (v_pk_fma_f32) peak, MI355X_MICROARCH.md
BF16_PEAK_TFLOPS = 2500.0  # dense bf16 MFMA (no sparsity), MI355X_MICROARCH.md


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--global-batch", type=int, default=512)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--lmax", type=int, default=10)
    ap.add_argument("--deconv-hidden", type=int, default=200)
    ap.add_argument("--mean-mode", default="s2s2")
    ap.add_argument("--channels-last", action="store_true")
    ap.add_argument("--amp", choices=["off", "bf16"], default="off",
                    help="bf16 autocast for the conv / deconv / linear layers (fp32 master "
                         "weights; the SO(3) kernels stay fp32)")
    ap.add_argument("--no-find", dest="find", action="store_false",
                    help="keep MIOpen's heuristic conv solutions (default: torch.backends."
                         "cudnn.benchmark, MIOpen times the candidates once per shape)")
    ap.add_argument("--conv-gemm", choices=["on", "off"], default="on",
                    help="run the two GEMM-shaped layers (decoder 1x1->4x4 ConvTranspose2d, "
                         "encoder 4x4->1x1 head) as addmm on hipBLASLt (on) or through MIOpen "
                         "(off); nets.GEMM_LAYERS")
    ap.add_argument("--deconv", choices=["transposed", "mfma"], default="mfma",
                    help="stride-2 ConvTranspose2d: MIOpen's transposed convolution or the "
                         "library's MFMA kernel for bf16 channels-last (nets.MFMA_DECONV)")
    ap.add_argument("--conv-dgrad", choices=["mfma", "miopen"], default="mfma",
                    help="encoder Conv2d(4, 2, 1) input gradients on the library's transposed-conv "
                         "kernel (nets.MFMA_CONV_DGRAD) or MIOpen")
    ap.add_argument("--adam", choices=["fused", "foreach"], default="fused",
                    help="torch.optim.Adam implementation (DPTrainer fused_adam)")
    ap.add_argument("--fused-relu", choices=["on", "off"], default="on",
                    help="DeconvNet's ReLUs inside the MFMA deconv kernels (nets.FUSED_RELU)")
    ap.add_argument("--graph", action="store_true",
                    help="capture the whole step (fwd, bwd, all-reduce, clip, Adam) in a "
                         "hipGraph and time its replays")
    ap.add_argument("--iwae", type=int, default=0, metavar="K",
                    help="time the IWAE log-likelihood (n=500) over K images instead")
    ap.add_argument("--iwae-n", type=int, default=500)
    ap.add_argument("--iwae-batch", type=int, default=8)
    ap.add_argument("--dry-run", action="store_true",
                    help="rehearse the rank plumbing on CPU (gloo, no HIP call)")
    args = ap.parse_args()
    env = launch.ensure_ranks(args.gpus, os.path.abspath(__file__))
    world, rank = env.world, env.rank
    if args.global_batch % world:
        raise SystemExit(f"global batch {args.global_batch} not divisible by {world} ranks")
    import torch.distributed as dist
    if args.dry_run:
        launch.init_process_group(env, "gloo")
        t = torch.tensor([float(rank)])
        if world > 1:
            dist.all_reduce(t)
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": world, "rank_sum": float(t.item()),
                              "per_gpu": args.global_batch // world}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return
    torch.backends.cudnn.benchmark = args.find
    if not args.find:  # immediate mode: off the package's find-db unless one is set
        from lie_vae.experiments import nets as _nets
        _nets.use_packaged_miopen_db()
    launch.init_process_group(env, "nccl")
    dev = torch.device("cuda", launch.device_index(env))
    torch.cuda.set_device(dev)

    from lie_vae.experiments import nets
    from lie_vae.experiments.vae import VAE
    nets.GEMM_LAYERS = args.conv_gemm == "on"
    nets.MFMA_DECONV = args.deconv == "mfma"
    nets.FUSED_RELU = args.fused_relu == "on"
    nets.MFMA_CONV_DGRAD = args.conv_dgrad == "mfma"

    torch.manual_seed(0)
    model = VAE(latent_mode="so3", decoder_mode="action", degrees=args.lmax, rep_copies=10,
                rgb=True, batch_norm=True, deconv_hidden=args.deconv_hidden,
                mean_mode=args.mean_mode).to(dev)
    if args.channels_last:
        model = model.to(memory_format=torch.channels_last)
    if args.iwae:
        return bench_iwae(args, model, env, dev)
    rec = time_train_steps(model, dev, world, rank, args.global_batch, args.steps, args.warmup,
                           amp=args.amp, graph=args.graph, fused_adam=args.adam == "fused")
    if rank == 0:
        rec["config"].update({"l_max": args.lmax, "deconv_hidden": args.deconv_hidden,
                              "mean_mode": args.mean_mode, "channels_last": args.channels_last,
                              "miopen_find": args.find, "conv_gemm": args.conv_gemm,
                              "deconv": args.deconv, "fused_relu": args.fused_relu,
                              "conv_dgrad": args.conv_dgrad, "adam": args.adam})
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


def _backend_name():
    """The process group's transport: 'nccl' is RCCL over xGMI on ROCm; gloo only in the
    one-GPU rehearsal (LV_SHARE_GPU0=1) and CPU tests."""
    import torch.distributed as dist
    b = dist.get_backend() if dist.is_initialized() else "none"
    return "RCCL (nccl backend)" if b == "nccl" else b


def time_train_steps(model, dev, world, rank, global_batch, steps, warmup, amp="off",
                     graph=False, fused_adam=True, flops=True, rounds=1):
    """Time `steps` DPTrainer steps (elbo fwd + bwd + bucketed all-reduce at world > 1 +
    global clip + Adam) on a synthetic per-rank shard after `warmup` steps; barrier +
    synchronize on both sides, max over ranks.  With rounds > 1 the timed loop runs that
    many times back to back and the record's time is the median round (every round's time
    is in the record): one stall of a few tens of ms inside a 40-ms window (seen once on a
    driver box: a 10.6 ms bf16 step against 3.9-4.3 ms in every rerun) no longer sets the
    figure.  Returns the record (rank 0 prints it)."""
    import torch.distributed as dist
    from lie_vae.experiments.train_dp import DPTrainer, param_count
    trainer = DPTrainer(model, lr=1e-3, clip_grads=1e-5,
                        amp_dtype=torch.bfloat16 if amp == "bf16" else None,
                        graph=graph, fused_adam=fused_adam)
    B = global_batch // world
    g = torch.Generator(device="cpu").manual_seed(100 + rank)
    x = torch.rand(B, 3, 64, 64, generator=g).to(dev)
    t_setup = time.perf_counter()
    for _ in range(warmup):
        trainer.step(x)
    step_flops = None
    if flops:
        # model FLOPs of one step (forward + backward, counted per aten op: the convs,
        # deconvs and linear layers; the SO(3) kernels are custom ops and not counted)
        from torch.utils.flop_counter import FlopCounterMode
        with FlopCounterMode(display=False) as fc:
            trainer.step(x)
        step_flops = fc.get_total_flops()
    run = trainer.capture(x) if graph else (lambda: trainer.step(x))
    torch.cuda.synchronize(dev)
    warm_s = time.perf_counter() - t_setup
    els, issue = [], []
    for _ in range(max(1, rounds)):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            loss, recon, kl = run()
        issue.append(time.perf_counter() - t0)  # host time to issue the steps
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        els.append(launch.max_over_ranks(time.perf_counter() - t0, dev))
    el = sorted(els)[len(els) // 2]
    nranks = launch.ranks_seen(dev)
    peak = F32_PEAK_TFLOPS if amp == "off" else BF16_PEAK_TFLOPS
    rec = {
        "metric": "VAE train samples/s (conv enc + SO(3) reparam + action dec, l=10)",
        "value": global_batch * steps / el, "unit": "samples/s", "n_gpus": world,
        "ranks_seen": nranks, "max_over_ranks": world > 1,
        "steps": steps, "warmup": warmup, "ms_per_step": el * 1e3 / steps,
        "rounds": max(1, rounds), "ms_per_step_rounds": [e * 1e3 / steps for e in els],
        # host time to issue a round's steps (rank 0): close to the round's time = host-bound
        "host_issue_ms_per_step_rounds": [e * 1e3 / steps for e in issue],
        "warmup_s": warm_s,
        "config": {"global_batch": global_batch, "per_gpu": B, "params": param_count(model),
                   "dtype": "f32" if amp == "off" else "bf16 autocast (convs/linear), f32 SO(3)",
                   "parallelism": (f"dp{world}: bucketed all-reduce of fp32 gradients over "
                                   f"{_backend_name()}" if world > 1 else "single GPU"),
                   "launch": "graph" if graph else "eager"},
        "loss": float(loss.item()), "recon": float(recon.mean().item()),
        "kl": float(kl.mean().item())}
    if step_flops is not None:
        rec["matrix"] = {"flops_per_step_per_gpu": step_flops,
                         "achieved_tflops_per_gpu": step_flops / (el / steps) / 1e12,
                         "peak_tflops": peak,
                         "frac": step_flops / (el / steps) / 1e12 / peak}
    return rec


def bench_iwae(args, model, env, dev):
    """IWAE evaluation throughput (images/s) at n = args.iwae_n: the reference's one-image
    calls, then args.iwae_batch images per call (same per-image terms)."""
    import torch.distributed as dist
    world, rank = env.world, env.rank
    # MIOpen's find on the n*B-image deconv shapes takes minutes per shape; the
    # evaluation runs each shape only K/B times, so it keeps the heuristic solutions
    torch.backends.cudnn.benchmark = False
    K = args.iwae // world
    g = torch.Generator(device="cpu").manual_seed(200 + rank)
    x = torch.rand(K, 3, 64, 64, generator=g).to(dev)
    model.eval()
    res = {}
    with torch.no_grad():
        for tag, bs in (("batch1", 1), (f"batch{args.iwae_batch}", args.iwae_batch)):
            for i in range(0, min(K, 2 * bs), bs):  # warm-up (MIOpen find per shape)
                model.log_likelihood(x[i:i + bs], n=args.iwae_n)
                torch.cuda.synchronize(dev)
                print(f"[iwae] {tag}: warm-up call done", file=sys.stderr, flush=True)
            if world > 1:
                dist.barrier()
            t0 = time.perf_counter()
            lls = [model.log_likelihood(x[i:i + bs], n=args.iwae_n) * x[i:i + bs].shape[0]
                   for i in range(0, K, bs)]
            ll = torch.stack(lls).sum()
            torch.cuda.synchronize(dev)
            el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
            if world > 1:
                dist.all_reduce(el, op=dist.ReduceOp.MAX)
                dist.all_reduce(ll)
            res[tag] = {"images_per_call": bs, "images_per_s": K * world / float(el.item()),
                        "ms_per_image": float(el.item()) * 1e3 / K,
                        "mean_ll": float(ll.item()) / (K * world)}
    if rank == 0:
        print(json.dumps({
            "metric": f"IWAE log-likelihood eval images/s (n={args.iwae_n})",
            "value": res[f"batch{args.iwae_batch}"]["images_per_s"], "unit": "images/s",
            "n_gpus": world, "images": K * world,
            "config": {"l_max": args.lmax, "deconv_hidden": args.deconv_hidden,
                       "mean_mode": args.mean_mode, "dtype": "f32",
                       "data": "synthetic x ~ U[0,1), random-init weights"},
            "runs": res}), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
