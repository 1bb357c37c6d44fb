"""Rank launcher of bench.py / bench_train.py (lie_vae/experiments/launch.py), on CPU.

``--gpus N`` without a torch.distributed environment must start N rank processes
(torch.distributed.run, rendezvous on 127.0.0.1) before any HIP call, and every rank
must see WORLD_SIZE = N; ``--dry-run`` runs the same control flow over gloo, so these
tests exercise the real hand-off without a GPU.  A WORLD_SIZE that contradicts
``--gpus`` must fail instead of timing fewer ranks than reported.
"""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=180):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "MASTER_ADDR")}
    env.update(env_extra or {})
    env["CUDA_VISIBLE_DEVICES"] = ""
    env["HIP_VISIBLE_DEVICES"] = ""
    p = subprocess.run([sys.executable, *args], cwd=REPO, env=env, capture_output=True,
                       text=True, timeout=timeout)
    return p


def _last_json(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert lines, out
    return json.loads(lines[-1])


@pytest.mark.parametrize("world", [1, 2])
def test_bench_spawns_ranks(world):
    p = _run(["bench.py", "--gpus", str(world), "--dry-run"])
    assert p.returncode == 0, p.stderr[-2000:]
    rec = _last_json(p.stdout)
    assert rec["dry_run"] is True
    assert rec["n_gpus"] == world
    assert rec["ranks_seen"] == world
    # exactly one JSON line (rank 0 only)
    assert sum(ln.startswith("{") for ln in p.stdout.splitlines()) == 1


def test_bench_train_spawns_ranks():
    p = _run(["bench_train.py", "--gpus", "2", "--global-batch", "4096", "--dry-run"])
    assert p.returncode == 0, p.stderr[-2000:]
    rec = _last_json(p.stdout)
    assert rec["n_gpus"] == 2 and rec["per_gpu"] == 2048
    assert rec["rank_sum"] == 1.0  # ranks 0 + 1 joined the all-reduce


def test_world_size_mismatch_fails():
    p = _run(["bench.py", "--gpus", "2", "--dry-run"],
             {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0
    assert "WORLD_SIZE" in (p.stderr + p.stdout)


def test_share_gpu0_rehearsal_mode(monkeypatch):
    """LV_SHARE_GPU0=1 (one-GPU rehearsal) binds every rank to cuda:0; by default each
    rank drives cuda:LOCAL_RANK."""
    sys.path.insert(0, os.path.join(REPO, "lie-vae_amd"))
    from lie_vae.experiments import launch
    env = launch.RankEnv(rank=3, local_rank=3, world=4)
    monkeypatch.delenv("LV_SHARE_GPU0", raising=False)
    assert launch.device_index(env) == 3 and not launch.share_gpu0()
    monkeypatch.setenv("LV_SHARE_GPU0", "1")
    assert launch.device_index(env) == 0 and launch.share_gpu0()
