"""One process per GPU for the benchmarks and the data-parallel trainer.

``python bench.py --gpus N`` (or ``bench_train.py``) started WITHOUT a torch.distributed
environment hands itself to ``torch.distributed.run`` (N fresh rank processes on this
node, rendezvous on 127.0.0.1) and exits with its status.  The hand-off happens before
anything touches HIP: the parent imports torch but never initialises a device, and the
ranks are started as CHILD processes (never exec'd over a process that initialised the
GPU).  Started by the driver's own ``torch.distributed.run`` (WORLD_SIZE set) the
script runs as that rank; a WORLD_SIZE that disagrees with ``--gpus`` is an error, so a
scaling run can never silently time fewer ranks than it reports.

The reference has no multi-device path at all (``lie_vae/experiments/main.py:17``);
this is the one-process-per-GPU layout of DESIGN.md §5.
"""
import os
import socket
import subprocess
import sys
from dataclasses import dataclass


@dataclass
class RankEnv:
    rank: int
    local_rank: int
    world: int

    @property
    def distributed(self):
        return self.world > 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def rank_env():
    return RankEnv(int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
                   int(os.environ.get("WORLD_SIZE", "1")))


def ensure_ranks(gpus, script, argv=None):
    """Return this process's RankEnv, or spawn ``gpus`` ranks of ``script`` and exit.

    Must be called before any HIP call in the process (``torch.cuda.is_available()``
    included)."""
    argv = list(sys.argv[1:] if argv is None else argv)
    if gpus < 1:
        raise SystemExit(f"--gpus must be >= 1 (got {gpus})")
    if "WORLD_SIZE" in os.environ:
        env = rank_env()
        if env.world != gpus:
            raise SystemExit(f"--gpus {gpus} but WORLD_SIZE={env.world}: launch with "
                             f"--nproc-per-node {gpus} or drop --gpus")
        return env
    if gpus == 1:
        return RankEnv(0, 0, 1)
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
           script, *argv]
    child_env = dict(os.environ)
    child_env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    rc = subprocess.call(cmd, env=child_env)
    raise SystemExit(rc)


def share_gpu0():
    """LV_SHARE_GPU0=1: rehearsal of the N-rank path on a one-GPU box -- every rank binds
    cuda:0 and the group runs over gloo (RCCL refuses two ranks on one device).  Off by
    default; never used for reported numbers."""
    return os.environ.get("LV_SHARE_GPU0", "0") == "1"


def device_index(env):
    """The GPU this rank drives: LOCAL_RANK (one process per GPU)."""
    return 0 if share_gpu0() else env.local_rank


def init_process_group(env, backend):
    """Bind cuda:LOCAL_RANK (nccl = RCCL on ROCm) and join the group; no-op at world 1."""
    import torch
    import torch.distributed as dist
    if backend == "nccl" and share_gpu0():
        torch.cuda.set_device(0)
        backend = "gloo"
    if backend == "nccl":
        torch.cuda.set_device(env.local_rank)
    if not env.distributed:
        return None
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", env.local_rank))
    else:
        dist.init_process_group(backend)
    return dist


def max_over_ranks(value, device=None):
    """Max of a float over all ranks (the benchmark's timing rule)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return float(value)
    if dist.get_backend() == "gloo":
        device = None
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def ranks_seen(device=None):
    """SUM all-reduce of a one from every rank over the live process group (RCCL under
    ``nccl``): the number of ranks the collective actually reached (1 without a group)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return 1
    if dist.get_backend() == "gloo":
        device = None
    t = torch.ones(1, dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(round(float(t.item())))
