#!/usr/bin/env python3
"""Benchmark of the SO(3) latent hot path on MI355X (BASELINE.json metric, config 2).

One step = one pass of the fused hot path (z = exp(v) -> ZYZ Euler -> block-diagonal
real Wigner-D(z) · F, l_max = 10, C = 10, fp32) over one batch of 4096 synthetic
samples already resident in HBM.  ``--gpus N`` runs one process per GPU: started
without a torch.distributed environment the script hands itself to
``torch.distributed.run`` before any HIP call (lie_vae/experiments/launch.py); started
by the driver's own ``torch.distributed.run`` it is that rank.  Every rank runs its
own 4096-sample batches: the path partitions by sample with no data-path collective,
so scaling is weak and the value is all ranks' samples / max-over-ranks time.  The
N = 1 output is unchanged by the launcher (no process group, no hand-off).

Prints ONE JSON line on rank 0 (contract in the task statement / DESIGN.md §6):
  value            samples/s, whole job
  roofline         HBM roofline of the fused kernel from live HIP-event timing (hot
                   Infinity Cache: back-to-back launches); ``cache_cold`` repeats it
                   with a 512 MiB scrub write between launches (> the 256 MiB MALL)
  cpu_baseline     the CPU oracle (reference op sequence, torch CPU) on a bounded
                   sample: all usable cores + 1 thread, forward and forward+backward
  fwd_bwd          the training direction on the GPU (fused forward + backward kernels)
  config5          BASELINE config 5 on every rank: l = 20, B = 8192 per GPU, bf16 out
                   (fp32 recursion), HBM and fp32-VALU roofline fractions
  train_step       BASELINE config 3 (N = 1: B = 512) / config 4 (N > 1: 512 per rank,
                   RCCL bucketed all-reduce of the gradients): the full VAE training step
                   (unsupervised.py:108-117) with bf16 autocast and at reference
                   precision (fp32; in that order), samples/s of the whole job, max over
                   ranks, the median of 3 timed rounds (each round's time in the record)
  fwd_bwd.*.roofline_valu  the group-action backward's VALU-issue roofline (it is VALU-bound
                   at large batch): PMC VALU instructions per call at the measured FMA
                   issue rate, as a fraction of the call time
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

from lie_vae.experiments import launch  # noqa: E402  (imports torch only; no HIP call)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table: 8.0 TB/s spec
F32_VALU_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: fp32 via v_pk_fma_f32 (= fp32 MFMA)
# The group-action backward is VALU-issue bound at large batch, so its records carry a VALU
# roofline next to the HBM one: the kernel's VALU wave-instructions per call (PMC
# SQ_INSTS_VALU of the backward kernel + its dF reduce, measured at HEAD with
# tools/gpu_pmc_bwd_only.sh) at the chip's measured scalar-FMA issue rate (661.19 wave
# instructions per ns = 3.72 cycles per instruction per SIMD, 8 waves per SIMD,
# tools/valu_rate.hip, profiles/r05_valu_rate.txt), as a fraction of the call time.
VALU_WAVE_INSTS_PER_NS = 661.19
BWD_VALU_PER_CALL = {  # batch -> (SQ_INSTS_VALU per call, evidence)
    4096: (2911261 + 51604, "profiles/r06_final_pmc_bwd_only_4096.txt"),
    65536: (40735328 + 51604, "profiles/r06_final_pmc_bwd_only_65536.txt"),
}
SCRUB_BYTES = 512 << 20  # > 256 MiB Infinity Cache (MI355X_MICROARCH.md:40)


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
    ap.add_argument("--events-in-graph", action="store_true",
                    help="record the timing events as nodes inside the first/last graph")
    ap.add_argument("--multistream", type=int, default=4,
                    help="also time this many independent batches in flight (extra field)")
    ap.add_argument("--cold-launches", type=int, default=40,
                    help="launches timed with a 512 MiB scrub between them (0: skip)")
    ap.add_argument("--cold-only", action="store_true",
                    help="only the scrubbed launches (for rocprofv3 kernel-trace runs)")
    ap.add_argument("--no-fwd-bwd", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=6.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--sweep", default="16384,65536",
                    help="comma-separated batches also timed (HIP events, median of 3 rounds); "
                         "'' to skip")
    ap.add_argument("--config5-launches", type=int, default=200,
                    help="config-5 record: launches timed per round (0: skip the record)")
    ap.add_argument("--train-steps", type=int, default=10,
                    help="train_step record: timed steps per precision (0: skip the record)")
    ap.add_argument("--train-warmup", type=int, default=10)
    ap.add_argument("--no-ang", action="store_true",
                    help="A/B only: time the instantiation without the angles output")
    ap.add_argument("--dry-run", action="store_true",
                    help="rehearse the rank plumbing on CPU (gloo, no HIP call)")
    return ap.parse_args()


def algorithmic_bytes(batch, L, C, out_bytes):
    """B·(in + M·C·sizeof(out)) + M·C·sizeof(F); in = 12 B (v)."""
    M = (L + 1) ** 2
    return batch * (12 + M * C * out_bytes) + M * C * 4


def workload_name(L, C, B, dtype):
    """BASELINE.json config the run matches (2: l=10, B=4096, fp32; 5: l=20, B=8192 per
    GPU, bf16 out), else the shape itself."""
    if (L, C, B, dtype) == (10, 10, 4096, "f32"):
        return "config2"
    if (L, C, B, dtype) == (20, 10, 8192, "bf16"):
        return "config5"
    return f"custom l={L} C={C} B={B} {dtype}"


def cpu_threads():
    """Threads for the CPU baseline: this process's affinity set, capped by the box's CPU
    share.  On the GPU box OMP_NUM_THREADS is the allotted share (16 of a 256-core host
    shared with other jobs' boxes); more threads would time oversubscribed cores, not the
    reference path, so the share is what "all usable cores" means there."""
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        usable = os.cpu_count() or 1
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return (min(usable, share) if share > 0 else usable), usable


def cpu_baseline(L, C, batch, seconds):
    """Reference op sequence on the host (oracle/lie_ref.py, a restatement of
    lie_tools.py:56-64,112-180,211-253), timed on a bounded sample of the benchmark's own
    batch (same B, l, C): forward on the usable cores and on 1 thread, forward+backward on
    the usable cores."""
    from oracle import lie_ref
    threads, usable = cpu_threads()
    g = torch.Generator().manual_seed(0)
    v = torch.randn(batch, 3, generator=g)
    F = torch.randn((L + 1) ** 2, C, generator=g)

    def fwd(vv, FF):
        ang = lie_ref.mat_to_eazyz(lie_ref.so3_exp(vv))
        return lie_ref.block_wigner_apply(ang, FF.expand(vv.shape[0], -1, -1), L)

    def timed(fn, budget, nb):
        fn()
        n, t0 = 0, time.perf_counter()
        while True:
            fn()
            n += 1
            el = time.perf_counter() - t0
            if el >= budget:
                return n * nb / el, n, el

    def fb():
        vg = v.clone().requires_grad_(True)
        Fg = F.clone().requires_grad_(True)
        fwd(vg, Fg).square().sum().backward()

    torch.set_num_threads(threads)
    with torch.no_grad():
        fw, nf, ef = timed(lambda: fwd(v, F), seconds, batch)
    fbw, nfb, efb = timed(fb, seconds, batch)
    torch.set_num_threads(1)
    with torch.no_grad():
        f1, n1, e1 = timed(lambda: fwd(v, F), seconds, batch)
    torch.set_num_threads(threads)
    return {"value": fw, "unit": "samples/s", "cores": threads, "kind": "port",
            "host_cores": os.cpu_count(), "usable_cores": usable,
            "cores_note": "OMP_NUM_THREADS share of the box (the GPU box allots 16 host "
                          "threads of a shared 256-core host); 1-thread figure alongside",
            "value_1thread": f1, "fwd_bwd_value": fbw,
            "sample": f"batch {batch} (exp+eazyz+action, l={L}, C={C}, fp32), torch CPU, "
                      f"oracle/lie_ref.py: forward {nf} batches in {ef:.1f}s on {threads} "
                      f"threads; forward+backward {nfb} batches in {efb:.1f}s on {threads} "
                      f"threads; forward {n1} batches in {e1:.1f}s on 1 thread"}


def dry_run(args, env):
    """Rank plumbing rehearsal on CPU: gloo group, barrier-bracketed timing, max over
    ranks, one JSON line from rank 0 -- the same control flow as the GPU run."""
    import torch.distributed as dist
    launch.init_process_group(env, "gloo")
    t0 = time.perf_counter()
    x = torch.ones(1)
    if env.distributed:
        dist.barrier()
        dist.all_reduce(x)
        dist.barrier()
    wall = launch.max_over_ranks(time.perf_counter() - t0)
    if env.rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": env.world, "ranks_seen": int(x.item()),
                          "local_rank": env.local_rank, "wall_s": wall}), flush=True)
    if env.distributed:
        dist.destroy_process_group()


def main():
    args = parse()
    env = launch.ensure_ranks(args.gpus, os.path.abspath(__file__))
    if args.dry_run:
        return dry_run(args, env)
    td = launch.init_process_group(env, "nccl")
    rank, world = env.rank, env.world
    dev = torch.device("cuda", launch.device_index(env))
    torch.cuda.set_device(dev)

    from lie_vae import _lib
    lib = _lib.load()
    L, C, B = args.lmax, args.channels, args.batch
    M = (L + 1) ** 2
    out_dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    dt = _lib.LV_DTYPE_BF16 if args.dtype == "bf16" else _lib.LV_DTYPE_F32
    out_bytes = 2 if args.dtype == "bf16" else 4
    abytes = algorithmic_bytes(B, L, C, out_bytes)
    g = torch.Generator(device="cpu").manual_seed(1000 + rank)
    v = torch.randn(B, 3, generator=g).to(dev)
    F = torch.randn(M, C, generator=g).to(dev)
    out = torch.empty(B, M, C, device=dev, dtype=out_dtype)
    # the product operator's instantiation writes the angles too (torch_ops.cpp,
    # lie_vae/_ops.py): the timed launches do the same (49 KB; not credited in the bytes)
    ang_buf = torch.empty(B, 3, device=dev)
    stream = torch.cuda.current_stream(dev)
    sp = ctypes.c_void_p(stream.cuda_stream)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731

    def launch_k(k, s=sp, o=None, vv=None, nb=B, a=None):
        o = out if o is None else o
        vv = v if vv is None else vv
        a = ang_buf if a is None else a
        rc = lib.lv_fused_exp_action_fwd_repeat(None, P(vv), P(F), 0, P(o), dt,
                                                None if args.no_ang else P(a), nb, L, C, 0, k, s)
        if rc:
            raise RuntimeError(_lib.last_error())

    def cold(nlaunch):
        """Per-launch kernel time with a 512 MiB scrub write between launches, so neither
        the output nor the inputs are resident in the 256 MiB Infinity Cache."""
        scrub = torch.empty(SCRUB_BYTES // 4, device=dev, dtype=torch.float32)
        evs = []
        for i in range(nlaunch + 2):
            scrub.fill_(float(i))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            launch_k(1)
            e1.record(stream)
            evs.append((e0, e1))
        torch.cuda.synchronize(dev)
        ts = sorted(e0.elapsed_time(e1) / 1e3 for e0, e1 in evs[2:])
        del scrub
        med = ts[len(ts) // 2]
        return {"launches": nlaunch, "us_median": med * 1e6, "us_min": ts[0] * 1e6,
                "achieved": abytes / med / 1e9, "frac": abytes / med / 1e9 / HBM_PEAK_GBS,
                "scrub_bytes": SCRUB_BYTES}

    if args.cold_only:
        rec = cold(max(1, args.cold_launches))
        if rank == 0:
            print(json.dumps({"cache_cold": rec}), flush=True)
        return

    # Timed region: K launches.  With --launch graph they are replayed from hipGraphs of
    # `chunk` launches, and the two timing events are nodes INSIDE the first and the last
    # graph (external event records): on a short region (the driver's 20 steps) events on
    # the stream around graph.replay() would also time the host's submission of the first
    # graph (~10 us before its first kernel starts), which is not kernel time.
    chunk = max(1, min(args.graph_chunk, args.steps))
    full, rem = divmod(args.steps, chunk)
    sizes = [chunk] * full + ([rem] if rem else [])
    events_in_graph = False  # set below once capture + replay proved they time the kernels
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    timed, warm_graph = [], None
    if args.launch == "graph":
        launch_k(1)
        torch.cuda.synchronize(dev)
        s = torch.cuda.Stream(dev)
        s.wait_stream(stream)
        cache = {}

        def graph_of(n, first, last):
            key = (n, first, last)
            if key not in cache:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=s):
                    if first:
                        ev0.record(s)
                    launch_k(n, ctypes.c_void_p(s.cuda_stream))
                    if last:
                        ev1.record(s)
                cache[key] = g
            return cache[key]

        warm_graph = graph_of(chunk, False, False)
        timed = [graph_of(n, False, False) for n in sizes]
        if args.events_in_graph:
            try:
                timed = [graph_of(n, i == 0, i == len(sizes) - 1) for i, n in enumerate(sizes)]
                events_in_graph = True
            except RuntimeError:
                timed = [graph_of(n, False, False) for n in sizes]
        torch.cuda.synchronize(dev)
        # the first replay of a fresh graph pays its one-time upload; every graph is
        # replayed once here, outside the timed region, whatever --warmup is
        for g in dict.fromkeys([warm_graph] + timed):
            g.replay()
        torch.cuda.synchronize(dev)

    def warmup_steps(k):
        if warm_graph is None:
            launch_k(k)
            return
        f, r = divmod(k, chunk)
        for _ in range(f):
            warm_graph.replay()
        if r:
            launch_k(r)

    warmup_steps(args.warmup)
    torch.cuda.synchronize(dev)
    if td:
        td.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if not events_in_graph:
        ev0.record(stream)
    if timed:
        for g in timed:
            g.replay()
    else:
        launch_k(args.steps)
    if not events_in_graph:
        ev1.record(stream)
    torch.cuda.synchronize(dev)
    if td:
        td.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    gpu_ms = ev0.elapsed_time(ev1)
    wall_max = launch.max_over_ranks(wall, dev)
    nranks = launch.ranks_seen(dev)  # after the timed region: ranks the collective reached

    value = B * args.steps * world / wall_max
    # The events around the timed region also hold a fixed cost that does not scale with
    # K: the first kernel's start after the idle, synchronised GPU (the host's submission
    # of the graph, the event packets).  It is ~8 us in total, i.e. +6% per launch at the
    # driver's K = 20 and nothing at K = 2000.  The same bracket around ONE launch
    # (median of 5, same graph/eager path, right after the timed region) measures it, and
    # the per-launch figure is the marginal (t_K - t_1) / (K - 1); the raw t_K / K is kept.
    raw_per_launch_s = gpu_ms / 1e3 / args.steps
    per_launch_s, t1_us = raw_per_launch_s, None
    if args.steps >= 10:
        # t_1 is bracketed exactly as t_K was: stream events around one replay, or (with
        # --events-in-graph) event nodes inside a one-launch graph
        if args.launch == "graph" and events_in_graph:
            g1 = graph_of(1, True, True)
        else:
            g1 = graph_of(1, False, False) if args.launch == "graph" else None
        if g1 is not None:
            g1.replay()
        ts = []
        for _ in range(5):
            torch.cuda.synchronize(dev)
            if events_in_graph:
                g1.replay()
                torch.cuda.synchronize(dev)
                ts.append(ev0.elapsed_time(ev1) / 1e3)
                continue
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            if g1 is not None:
                g1.replay()
            else:
                launch_k(1)
            e1.record(stream)
            torch.cuda.synchronize(dev)
            ts.append(e0.elapsed_time(e1) / 1e3)
        t1 = sorted(ts)[2]
        t1_us = t1 * 1e6
        per_launch_s = (gpu_ms / 1e3 - t1) / (args.steps - 1)
    achieved = abytes / per_launch_s / 1e9

    sweep = None
    sweep_batches = [int(b) for b in args.sweep.split(",") if b.strip()]
    if sweep_batches and rank == 0:
        sweep = []
        for nb in sweep_batches:
            vv = torch.randn(nb, 3, device=dev)
            oo = torch.empty(nb, M, C, device=dev, dtype=out_dtype)
            aa = torch.empty(nb, 3, device=dev)
            # >= ~10 ms of launches per round: the first rounds after a fresh output
            # allocation run up to 30% slow (tools/sweep_dist.py), so one untimed round,
            # then the median of three
            reps = max(50, int(2e5 // nb) * 50)
            ts = []
            for it in range(4):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                launch_k(reps, o=oo, vv=vv, nb=nb, a=aa)
                e1.record(stream)
                torch.cuda.synchronize(dev)
                if it:
                    ts.append(e0.elapsed_time(e1) / 1e3 / reps)
            t = sorted(ts)[1]
            gbs = algorithmic_bytes(nb, L, C, out_bytes) / t / 1e9
            sweep.append({"batch": nb, "us": t * 1e6, "GB/s": gbs, "frac": gbs / HBM_PEAK_GBS})
            del vv, oo, aa

    # independent batches on parallel streams (same kernel): aggregate throughput
    multi = None
    if args.launch == "graph" and args.multistream > 1:
        ms = args.multistream
        mouts = [torch.empty(B, M, C, device=dev, dtype=out_dtype) for _ in range(ms)]
        mangs = [torch.empty(B, 3, device=dev) for _ in range(ms)]
        side = [torch.cuda.Stream(dev) for _ in range(ms)]
        mchunk = max(ms, chunk - chunk % ms)
        g2 = torch.cuda.CUDAGraph()
        s2 = torch.cuda.Stream(dev)
        s2.wait_stream(stream)
        with torch.cuda.graph(g2, stream=s2):
            for t in side:
                t.wait_stream(s2)
            for t, o, a in zip(side, mouts, mangs):
                launch_k(mchunk // ms, ctypes.c_void_p(t.cuda_stream), o, a=a)
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
        del mouts, mangs

    cache_cold = cold(args.cold_launches) if args.cold_launches > 0 and rank == 0 else None

    fwd_bwd = None
    if not args.no_fwd_bwd and rank == 0 and args.dtype == "f32":
        fwd_bwd = bench_fwd_bwd(v, F, L, dev, stream)

    # HBM traffic per launch is NOT measured in this run (PMC counters need their own
    # rocprofv3 --pmc passes, tools/gpu_prof.sh): it is read from the committed summary of
    # those passes for this exact shape, and the line says so ("traffic_source")
    traffic, traffic_source = None, None
    tname = f"traffic_B{B}_L{L}_C{C}_{args.dtype}.json"
    tpath = os.path.join(REPO, "profiles", tname)
    if os.path.exists(tpath):
        with open(tpath) as f:
            tj = json.load(f)
        traffic = tj.get("hbm_bytes_per_launch")
        traffic_source = (f"profiles/{tname}: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes "
                          f"({tj.get('measured', 'committed earlier')}), read from the file, not "
                          "measured in this run")

    # BASELINE configs 5 and 3 / 4 as bounded sub-records of the same line (every rank
    # takes part: they are timed max over ranks like the headline)
    config5 = None
    if args.config5_launches > 0:
        config5 = bench_config5(lib, dev, stream, world, rank, args.config5_launches)
    train = None
    if args.train_steps > 0:
        train = bench_train_step(dev, env, args.train_steps, args.train_warmup)

    # the CPU baseline last: ~18 s of all-thread host work right before the host-bound
    # bf16 training step slowed that step 1.2-2.7x on the driver's box (3.9-4.3 ms per step
    # without it in the same bench, 4.8-10.6 ms after it)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(L, C, B, args.cpu_seconds)

    if rank == 0:
        rec = {
            "metric": f"SO(3) samples/sec (exp+WignerD+action, l_max={L})",
            "value": value,
            "unit": "samples/s",
            "n_gpus": world,
            "ranks_seen": nranks,
            "max_over_ranks": world > 1,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": wall_max * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32" if args.dtype == "f32" else "f32 compute, bf16 out",
            "data": "synthetic: v ~ N(0,1)^(Bx3) per rank (seeded), F ~ N(0,1)^((L+1)^2 x C)",
            "config": {"workload": f"{workload_name(L, C, B, args.dtype)}: fused exp -> ZYZ -> "
                                   "block Wigner-D action (lv_fused_exp_action_fwd)",
                       "batch_per_gpu": B, "global_batch": B * world, "l_max": L,
                       "channels": C, "parallelism": f"sample-sharded x{world}, no collective",
                       "launch": args.launch},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_source": traffic_source,
                         "algorithmic_bytes_per_launch": abytes,
                         "us_per_launch_events": per_launch_s * 1e6,
                         "us_per_launch_events_raw": raw_per_launch_s * 1e6,
                         "us_one_launch_bracket": t1_us,
                         "per_launch_rule": "MARGINAL per-launch time (t_K - t_1) / (K - 1): "
                                            "HIP events bracket the K timed launches and, the "
                                            "same way, one launch (median of 5); the fixed "
                                            "submission cost both brackets hold cancels. The "
                                            "raw t_K / K is us_per_launch_events_raw",
                         "events": "graph nodes" if events_in_graph else "stream",
                         "instantiation": ("A/B: no angles output" if args.no_ang else
                                           "product (angles written, as torch.ops.lievae."
                                           "fused_exp_action)"),
                         "cache": "hot (back-to-back launches)"},
            "cache_cold": cache_cold,
            "cpu_baseline": cpu,
            "fwd_bwd": fwd_bwd,
            "multistream": multi,
            "sweep": sweep,
            "config5": config5,
            "train_step": train,
        }
        print(json.dumps(rec), flush=True)
    if td:
        td.destroy_process_group()


def bench_config5(lib, dev, stream, world, rank, launches, L=20, C=10, B=8192):
    """BASELINE config 5: the fused exp -> ZYZ -> Wigner-D action at l = 20, B = 8192 per
    GPU, bf16 output with fp32 recursion (lv_fused_exp_action_fwd, dtype bf16, writing the
    angles as the product operator does).  Every rank times `launches` back-to-back launches
    (HIP events on the launch stream, median of 3 rounds after an untimed one); the barrier
    brackets the rounds and the value is all ranks' samples / the max-over-ranks time.
    Roofline: HBM on the algorithmic bytes (72,369,384 B per launch) and
    fp32 VALU on the D·F FLOPs (2·C·S_D = 246,820 per sample; the recursion's FLOPs are
    implementation-dependent and not credited)."""
    import torch.distributed as dist
    M = (L + 1) ** 2
    S_D = (L + 1) * (2 * L + 1) * (2 * L + 3) // 3
    g = torch.Generator(device="cpu").manual_seed(5000 + rank)
    v = torch.randn(B, 3, generator=g).to(dev)
    F = torch.randn(M, C, generator=g).to(dev)
    out = torch.empty(B, M, C, device=dev, dtype=torch.bfloat16)
    ang = torch.empty(B, 3, device=dev)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    sp = ctypes.c_void_p(stream.cuda_stream)

    def run(k):
        rc = lib.lv_fused_exp_action_fwd_repeat(None, P(v), P(F), 0, P(out), 1, P(ang), B, L, C,
                                                0, k, sp)
        if rc:
            raise RuntimeError("lv_fused_exp_action_fwd (config 5) failed")

    run(2)
    torch.cuda.synchronize(dev)
    if dist.is_initialized():
        dist.barrier()
    t0 = time.perf_counter()
    ts = []
    for it in range(4):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        run(launches)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        if it:
            ts.append(e0.elapsed_time(e1) / 1e3 / launches)
    if dist.is_initialized():
        dist.barrier()
    wall = time.perf_counter() - t0
    us = sorted(ts)[1] * 1e6
    us_max = max(ts) * 1e6
    from lie_vae.experiments import launch as _launch
    us_all = _launch.max_over_ranks(us, dev)
    abytes = algorithmic_bytes(B, L, C, 2)
    flops = 2 * C * S_D * B
    hbm = abytes / (us_all * 1e-6) / 1e9
    tf = flops / (us_all * 1e-6) / 1e12
    return {"workload": "config5: fused exp -> ZYZ -> block Wigner-D action, l=20, C=10, "
                        "B=8192 per GPU, bf16 out, fp32 recursion and angles",
            "value": B * world / (us_all * 1e-6), "unit": "samples/s", "n_gpus": world,
            "us_per_launch": us_all, "us_per_launch_rank0_median": us, "us_rank0_worst": us_max,
            "launches_per_round": launches, "rounds_timed": 3, "wall_s": wall,
            "timing": "HIP events around `launches` back-to-back launches on the launch "
                      "stream, median of 3 rounds, max over ranks",
            "roofline_hbm": {"achieved": hbm, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": hbm / HBM_PEAK_GBS, "algorithmic_bytes_per_launch": abytes},
            "roofline_valu_f32": {"achieved": tf, "peak": F32_VALU_PEAK_TFLOPS,
                                  "unit": "TFLOP/s", "frac": tf / F32_VALU_PEAK_TFLOPS,
                                  "flops_per_launch": flops,
                                  "flops_note": "D·F only, 2·C·S_D per sample (S_D = 12,341)"}}


def bench_train_step(dev, env, steps, warmup):
    """BASELINE config 3 (N = 1: batch 512) and config 4 (N > 1: 512 per rank, the global
    batch 512·N, RCCL bucketed all-reduce of the fp32 gradients, global-norm clip, Adam):
    the reference's training step (unsupervised.py:108-117, VAE so3 / action, l = 10,
    C = 10, deconv_hidden 200, s2s2 mean, batch norm, RGB 64x64) on synthetic x ~ U[0,1)
    resident in HBM and random-init weights.  Twice: at the reference's fp32 and with bf16
    autocast on the conv / linear layers (channels-last; the SO(3) kernels stay fp32).
    MIOpen runs in immediate mode (no find) off the package's find-db
    (lie_vae/data/miopen, nets.use_packaged_miopen_db)."""
    import bench_train
    from lie_vae.experiments import nets
    from lie_vae.experiments.vae import VAE
    db = nets.use_packaged_miopen_db()
    torch.backends.cudnn.benchmark = False
    # the buffers of the records before (sweep, cold-cache scrub, config 5) back to the
    # device: the step's allocations then come from fresh segments, as in a training
    # process (bench_train.py alone: 3.80 ms bf16; after them without this, 4.0-5.8)
    import gc
    gc.collect()
    torch.cuda.empty_cache()
    recs = {}
    t0 = time.perf_counter()
    # bf16 first: right after the fp32 step's 100 TFLOP/s fp32-MFMA layers its first rounds
    # ran 20-30% slow (5.46 / 5.33 / 4.37 ms against 3.8-4.0 in steady state)
    for tag, amp, cl in (("bf16", "bf16", True), ("f32", "off", False)):
        torch.manual_seed(0)
        model = VAE(latent_mode="so3", decoder_mode="action", degrees=10, rep_copies=10,
                    rgb=True, batch_norm=True, deconv_hidden=200, mean_mode="s2s2").to(dev)
        if cl:
            model = model.to(memory_format=torch.channels_last)
        rec = bench_train.time_train_steps(model, dev, env.world, env.rank, 512 * env.world,
                                           steps, warmup, amp=amp, rounds=3)
        rec["config"]["channels_last"] = cl
        recs[tag] = rec
        del model
        torch.cuda.empty_cache()
    recs["workload"] = (("config4: " if env.world > 1 else "config3: ") +
                        "full sphere-cube VAE training step, 512 images per GPU")
    recs["wall_s"] = time.perf_counter() - t0
    recs["data"] = "synthetic x ~ U[0,1)^(512x3x64x64) per rank (seeded), random-init weights"
    recs["miopen"] = ("immediate mode, find-db " + ("lie_vae/data/miopen (tools/gen_miopen_db.sh)"
                                                    if db else "absent: fallback heuristics"))
    return recs


def bench_fwd_bwd(v, F, L, dev, stream, iters=200):
    """Training direction at the metric size: the fused forward and the full backward
    (group-action backward kernel + dF reduce + exp -> ZYZ VJP) through the autograd ops,
    (a) eager (host launch overhead included) and (b) the same forward + backward
    captured once in a hipGraph and replayed (whole-step capture, static tensors)."""
    import lie_vae._ops as ops
    B, C = v.shape[0], F.shape[1]
    vg = v.clone().requires_grad_(True)
    Fg = F.clone().requires_grad_(True)
    gout = torch.randn(B, (L + 1) ** 2, C, device=dev)

    def step():
        vg.grad = None
        Fg.grad = None
        out = ops.fused_exp_action(None, vg, Fg, L)
        out.backward(gout)

    for _ in range(5):
        step()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(iters):
        step()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    t = e0.elapsed_time(e1) / 1e3 / iters
    # (b) graph-captured forward + backward
    side = torch.cuda.Stream(dev)
    side.wait_stream(stream)
    with torch.cuda.stream(side):
        for _ in range(3):
            step()
    stream.wait_stream(side)
    torch.cuda.synchronize(dev)
    g = torch.cuda.CUDAGraph()
    vg.grad = None
    Fg.grad = None
    with torch.cuda.graph(g):
        out = ops.fused_exp_action(None, vg, Fg, L)
        out.backward(gout)
    g.replay()
    torch.cuda.synchronize(dev)
    reps = 500
    e0.record(stream)
    for _ in range(reps):
        g.replay()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    tg = e0.elapsed_time(e1) / 1e3 / reps
    kern = bench_action_bwd_kernel(vg.detach(), F, gout, L, dev)
    kern_fused = bench_action_bwd_kernel(vg.detach(), F, gout, L, dev, fused=True)
    # the large-batch backward (persistent kernel, action_bwd_persist.h) at 65,536 samples
    g2 = torch.Generator(device="cpu").manual_seed(77)
    vb = torch.randn(65536, 3, generator=g2).to(dev)
    gb = torch.randn(65536, (L + 1) ** 2, C, generator=g2).to(dev)
    kern_big = bench_action_bwd_kernel(vb, F, gb, L, dev, reps=200)
    del vb, gb
    return {"value": B / tg, "unit": "samples/s", "us_per_step": tg * 1e6,
            "launch": "graph (forward + backward captured once, replayed)",
            "eager_us_per_step": t * 1e6, "eager_value": B / t,
            "action_bwd": kern, "action_bwd_fused": kern_fused,
            "action_bwd_65536": kern_big,
            "note": "one training-direction pass: fused forward, group-action backward "
                    "kernel + deterministic dF reduce + fused exp/ZYZ VJP"}


def bench_action_bwd_kernel(v, F, gout, L, dev, reps=200, fused=False):
    """lv_group_action_bwd alone (backward tile kernel + deterministic dF reduce), graph-
    captured back-to-back calls on resident inputs: the angle/spectrum gradient of
    block_wigner_matrix_multiply (lie_tools.py:226-253) at the metric size.  fused=True:
    lv_fused_exp_action_bwd, the training path (the same kernels, the exp -> ZYZ VJP beside
    the reduce; v -> gv instead of the angle gradient)."""
    import lie_vae._ops as ops
    from lie_vae import _lib
    lib = _lib.load()
    B, C = v.shape[0], F.shape[1]
    M = (L + 1) ** 2
    ang = torch.empty(B, 3, device=dev)
    out = ops.fused_exp_action(None, v, F, L)
    lib.lv_fused_exp_action_fwd(None, ctypes.c_void_p(v.data_ptr()), ctypes.c_void_p(F.data_ptr()), 0,
                                ctypes.c_void_p(out.data_ptr()), _lib.LV_DTYPE_F32,
                                ctypes.c_void_p(ang.data_ptr()), B, L, C, 0, None)
    gang = torch.empty(B, 3, device=dev)
    gv = torch.empty(B, 3, device=dev)
    gF = torch.empty(M, C, device=dev)
    ws_bytes = lib.lv_group_action_bwd_workspace(B, L, C, 1)
    ws = torch.empty(max(ws_bytes, 1), device=dev, dtype=torch.uint8)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    torch.cuda.synchronize(dev)
    s = torch.cuda.Stream(dev)

    def call(k, st):
        for _ in range(k):
            if fused:
                rc = lib.lv_fused_exp_action_bwd(None, P(v), P(ang), P(F), P(gout), None, P(gv), P(gF),
                                                 B, L, C, 0, P(ws), ws_bytes, ctypes.c_void_p(st.cuda_stream))
            else:
                rc = lib.lv_group_action_bwd(P(ang), P(F), 0, P(gout), P(gang), P(gF), B, L, C, 0,
                                             P(ws), ws_bytes, ctypes.c_void_p(st.cuda_stream))
            if rc:
                raise RuntimeError(_lib.last_error())

    call(2, s)
    torch.cuda.synchronize(dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        call(50, s)
    g.replay()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    cur = torch.cuda.current_stream(dev)
    e0.record(cur)
    for _ in range(reps // 50):
        g.replay()
    e1.record(cur)
    torch.cuda.synchronize(dev)
    us = e0.elapsed_time(e1) * 1e3 / (reps // 50 * 50)
    plan = _lib.plan("bwd", B, L, C, 1)
    slab_bytes = plan["blocks"] * (-(-M * C // 16) * 16) * 4
    bb = B * (12 + M * C * 4 + 12) + 2 * M * C * 4 + slab_bytes * 2
    bmin = B * (12 + M * C * 4 + 12) + 2 * M * C * 4
    valu = None
    if not fused and B in BWD_VALU_PER_CALL:
        insts, src = BWD_VALU_PER_CALL[B]
        issue_us = insts / VALU_WAVE_INSTS_PER_NS / 1e3
        valu = {"bound": "valu", "valu_wave_insts_per_call": insts, "issue_us": issue_us,
                "rate_wave_insts_per_ns": VALU_WAVE_INSTS_PER_NS, "frac": issue_us / us,
                "source": src + " (PMC) / profiles/r05_valu_rate.txt (issue rate)"}
    return {"us_per_call": us, "roofline_valu": valu, "batch": B, "samples_per_s": B / us * 1e6, "bytes_per_call": bb,
            "achieved_GBs": bb / us / 1e3, "frac": bb / us / 1e3 / HBM_PEAK_GBS,
            "min_bytes_per_call": bmin, "frac_min_bytes": bmin / us / 1e3 / HBM_PEAK_GBS,
            "kernel": ("persistent (action_bwd_persist_kernel)" if plan["tile"] == 3 else
                       "one group per block (action_bwd_tile_kernel)") +
                      (" + reduce5 with the exp -> ZYZ VJP beside it (lv_fused_exp_action_bwd)" if fused else ""),
            "blocks": plan["blocks"],
            "bytes_note": "angles + output gradient in, angle gradient out, F in / dF out, "
                          "the dF slabs written and read once (one per block); "
                          "min_bytes_per_call leaves the slabs out"}


if __name__ == "__main__":
    main()
