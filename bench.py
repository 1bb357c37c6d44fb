#!/usr/bin/env python3
"""Benchmark of the SO(3) latent hot path on MI355X (BASELINE.json metric, config 2).

One step = one pass of the fused hot path (z = exp(v) -> ZYZ Euler -> block-diagonal
real Wigner-D(z) · F, l_max = 10, C = 10, fp32) over one batch of 4096 synthetic
samples already resident in HBM.  With --gpus N (one process per GPU, launched by
torch.distributed.run) every rank runs its own 4096-sample batches: the path
partitions by sample with no data-path collective, so scaling is weak and the
value is the sum over ranks (all-rank samples / max-over-ranks time).

Prints ONE JSON line on rank 0 (contract in the task statement / DESIGN.md §Bench):
  value            samples/s, whole job
  roofline         HBM roofline of the fused kernel from live HIP-event timing
  cpu_baseline     the CPU oracle (reference op sequence, torch CPU) on a bounded sample
"""
import argparse
import ctypes
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "lie-vae_amd"))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table: 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--lmax", type=int, default=10)
    ap.add_argument("--channels", type=int, default=10)
    ap.add_argument("--dtype", choices=["f32", "bf16"], default="f32")
    ap.add_argument("--launch", choices=["graph", "eager"], default="graph",
                    help="graph: steps captured in a hipGraph and replayed; eager: C launch loop")
    ap.add_argument("--graph-chunk", type=int, default=100)
    ap.add_argument("--streams", type=int, default=1,
                    help="independent batches in flight on this many HIP streams (graph mode)")
    ap.add_argument("--multistream", type=int, default=4,
                    help="also time this many independent batches in flight (extra field)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--sweep", action="store_true", help="also print a batch sweep (stderr)")
    return ap.parse_args()


def algorithmic_bytes(batch, L, C, out_bytes):
    """B·(in + M·C·sizeof(out)) + M·C·sizeof(F); in = 12 B (v)."""
    M = (L + 1) ** 2
    return batch * (12 + M * C * out_bytes) + M * C * 4


def cpu_baseline(L, C, batch, seconds):
    """Reference op sequence on the host (oracle/lie_ref.py), timed on a bounded sample."""
    from oracle import lie_ref
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(0)
    v = torch.randn(batch, 3, generator=g)
    F = torch.randn((L + 1) ** 2, C, generator=g)
    with torch.no_grad():
        def run():
            ang = lie_ref.mat_to_eazyz(lie_ref.so3_exp(v))
            return lie_ref.block_wigner_apply(ang, F.expand(batch, -1, -1), L)
        run()
        n, t0 = 0, time.perf_counter()
        while True:
            run()
            n += 1
            el = time.perf_counter() - t0
            if el >= seconds:
                break
    return {"value": n * batch / el, "unit": "samples/s", "cores": threads, "kind": "port",
            "sample": f"{n} batches x {batch} samples (exp+eazyz+action, l={L}, C={C}, fp32) "
                      f"in {el:.1f}s, torch CPU, {threads} threads"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    if dist:
        import torch.distributed as td
        torch.cuda.set_device(local)
        td.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from lie_vae import _lib
    lib = _lib.load()
    L, C, B = args.lmax, args.channels, args.batch
    M = (L + 1) ** 2
    out_dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    dt = _lib.LV_DTYPE_BF16 if args.dtype == "bf16" else _lib.LV_DTYPE_F32
    g = torch.Generator(device="cpu").manual_seed(1000 + rank)
    v = torch.randn(B, 3, generator=g).to(dev)
    F = torch.randn(M, C, generator=g).to(dev)
    nstreams = max(1, args.streams if args.launch == "graph" else 1)
    outs = [torch.empty(B, M, C, device=dev, dtype=out_dtype) for _ in range(nstreams)]
    out = outs[0]
    stream = torch.cuda.current_stream(dev)
    sp = ctypes.c_void_p(stream.cuda_stream)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731

    def launch(k, s=sp, o=None):
        o = out if o is None else o
        rc = lib.lv_fused_exp_action_fwd_repeat(None, P(v), P(F), 0, P(o), dt, None, B, L, C, 0,
                                                k, s)
        if rc:
            raise RuntimeError(_lib.last_error())

    graph = None
    chunk = max(1, min(args.graph_chunk, args.steps))
    if args.launch == "graph":
        launch(1)
        torch.cuda.synchronize(dev)
        s = torch.cuda.Stream(dev)
        s.wait_stream(stream)
        graph = torch.cuda.CUDAGraph()
        if nstreams > 1:
            chunk = max(nstreams, chunk - chunk % nstreams)
            side = [torch.cuda.Stream(dev) for _ in range(nstreams)]
        with torch.cuda.graph(graph, stream=s):
            if nstreams == 1:
                launch(chunk, ctypes.c_void_p(s.cuda_stream))
            else:  # fork: independent batches on parallel graph branches, then join
                for t in side:
                    t.wait_stream(s)
                for t, o in zip(side, outs):
                    launch(chunk // nstreams, ctypes.c_void_p(t.cuda_stream), o)
                for t in side:
                    s.wait_stream(t)
        torch.cuda.synchronize(dev)

    def run_steps(k):
        if graph is None:
            launch(k)
            return
        full, rem = divmod(k, chunk)
        for _ in range(full):
            graph.replay()
        if rem:
            launch(rem)

    run_steps(args.warmup)
    torch.cuda.synchronize(dev)
    if dist:
        td.barrier()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(torch.cuda.current_stream(dev))
    run_steps(args.steps)
    ev1.record(torch.cuda.current_stream(dev))
    torch.cuda.synchronize(dev)
    if dist:
        td.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    gpu_ms = ev0.elapsed_time(ev1)
    el = torch.tensor([wall], dtype=torch.float64, device=dev)
    if dist:
        td.all_reduce(el, op=td.ReduceOp.MAX)
    wall_max = float(el.item())

    samples = B * args.steps * world
    value = samples / wall_max
    per_launch_s = gpu_ms / 1e3 / args.steps
    out_bytes = 2 if args.dtype == "bf16" else 4
    abytes = algorithmic_bytes(B, L, C, out_bytes)
    achieved = abytes / per_launch_s / 1e9

    sweep = []
    if args.sweep and rank == 0:
        for nb in (4096, 16384, 65536, 262144):
            vv = torch.randn(nb, 3, device=dev)
            oo = torch.empty(nb, M, C, device=dev, dtype=out_dtype)
            for rep in range(2):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                reps = 50
                e0.record()
                rc = lib.lv_fused_exp_action_fwd_repeat(None, P(vv), P(F), 0, P(oo), dt, None, nb,
                                                        L, C, 0, reps, sp)
                e1.record()
                torch.cuda.synchronize(dev)
            t = e0.elapsed_time(e1) / 1e3 / reps
            gbs = algorithmic_bytes(nb, L, C, out_bytes) / t / 1e9
            sweep.append({"batch": nb, "us": t * 1e6, "GB/s": gbs, "frac": gbs / HBM_PEAK_GBS})
            del vv, oo
        print(json.dumps({"sweep": sweep}), file=sys.stderr)

    # independent batches on parallel streams (same kernel): aggregate throughput
    multi = None
    if args.launch == "graph" and nstreams == 1 and args.multistream > 1:
        ms = args.multistream
        mouts = [torch.empty(B, M, C, device=dev, dtype=out_dtype) for _ in range(ms)]
        side = [torch.cuda.Stream(dev) for _ in range(ms)]
        mchunk = max(ms, chunk - chunk % ms)
        g2 = torch.cuda.CUDAGraph()
        s2 = torch.cuda.Stream(dev)
        s2.wait_stream(stream)
        with torch.cuda.graph(g2, stream=s2):
            for t in side:
                t.wait_stream(s2)
            for t, o in zip(side, mouts):
                launch(mchunk // ms, ctypes.c_void_p(t.cuda_stream), o)
            for t in side:
                s2.wait_stream(t)
        reps = max(1, args.steps // mchunk)
        for _ in range(2):
            g2.replay()
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        for _ in range(reps):
            g2.replay()
        torch.cuda.synchronize(dev)
        el2 = time.perf_counter() - t1
        multi = {"streams": ms, "steps": reps * mchunk, "value": reps * mchunk * B * world / el2,
                 "unit": "samples/s", "us_per_step": el2 / (reps * mchunk) * 1e6,
                 "aggregate_GBs": abytes * reps * mchunk / el2 / 1e9}
        del mouts

    traffic = None
    tpath = os.path.join(REPO, "profiles", f"traffic_B{B}_L{L}_C{C}_{args.dtype}.json")
    if os.path.exists(tpath):
        traffic = json.load(open(tpath)).get("hbm_bytes_per_launch")

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(L, C, B, args.cpu_seconds)

    if rank == 0:
        rec = {
            "metric": "SO(3) samples/sec (exp+WignerD+action, l_max=10)",
            "value": value,
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": wall_max * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32" if args.dtype == "f32" else "f32 compute, bf16 out",
            "data": "synthetic: v ~ N(0,1)^(Bx3) per rank (seeded), F ~ N(0,1)^((L+1)^2 x C)",
            "config": {"workload": "config2: fused exp -> ZYZ -> block Wigner-D action "
                                   "(lv_fused_exp_action_fwd)",
                       "batch_per_gpu": B, "global_batch": B * world, "l_max": L,
                       "channels": C, "parallelism": f"sample-sharded x{world}, no collective",
                       "launch": args.launch, "streams": nstreams},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "algorithmic_bytes_per_launch": abytes,
                         "us_per_launch_events": per_launch_s * 1e6},
            "cpu_baseline": cpu,
            "multistream": multi,
        }
        print(json.dumps(rec), flush=True)
    if dist:
        td.destroy_process_group()


if __name__ == "__main__":
    main()
