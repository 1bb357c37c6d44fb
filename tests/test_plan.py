"""Host launch planning of the group-action kernels (action.hip plan_fwd / plan_bwd),
through the host-only C-ABI entries lv_action_fwd_plan / lv_group_action_bwd_plan: no
GPU call, so this runs on CPU.  The invariants are what the kernels assume about their
grid and LDS (action_fwd.h, action_bwd.h); a plan that broke one would fault the GPU."""
import pytest

from lie_vae import _lib

LDS_PER_CU = 160 * 1024
TILE_MAX_LDS = 80 * 1024       # action.hip kTileMaxLds
BWD_MAX_LDS = 96 * 1024        # action.hip kBwdMaxLds
BWD_MAX_BLOCKS = 4096          # action.hip kBwdMaxBlocks
CUS = _lib.load().lv_compute_units()  # the planner's CU count (256 on MI355X / no device)
PERSIST_BLOCKS = 3 * CUS                # action_bwd_persist.h kBwdPersistBlocksPerCU
PERSIST_MIN_GROUPS = CUS + 1            # persistent kernel beyond one group per CU
F32, BF16 = _lib.LV_DTYPE_F32, _lib.LV_DTYPE_BF16
NS = (1, 5, 6, 7, 683, 4096, 8192, 65536, 1 << 20)


def _check_segments(p, L):
    seg = p["seg_lo"]
    assert len(seg) == p["segments"] + 1
    assert seg[0] == 0 and seg[-1] == L + 1
    assert all(a < b for a, b in zip(seg, seg[1:])), seg
    # the degree sets the kernels run: one non-empty set per wave, together a partition of
    # 0..L (each degree's rows belong to exactly one wave)
    masks = p["seg_mask"]
    assert len(masks) == p["segments"] and all(m > 0 for m in masks), masks
    acc = 0
    for m in masks:
        assert acc & m == 0, masks
        acc |= m
    assert acc == (1 << (L + 1)) - 1, masks


@pytest.mark.parametrize("L", list(range(0, 21)))
def test_forward_plans_fit_the_kernels(L):
    for C in (1, 3, 10, 16, 64):
        M = (L + 1) ** 2
        for n in NS:
            for fused, fstride, dt in ((1, 0, F32), (1, 0, BF16), (0, 0, F32), (0, 0, BF16),
                                       (0, M * C, F32)):
                p = _lib.plan("fwd", fused, fstride, dt, n, L, C)
                _check_segments(p, L)
                assert p["samples_per_group"] == 64 // C
                assert p["lds_bytes"] <= LDS_PER_CU
                assert p["threads"] <= 1024 and p["threads"] % 64 == 0
                if p["tile"]:
                    assert fstride == 0
                    # __launch_bounds__(512); the prologue needs 3 threads per sample
                    assert p["threads"] == 64 * p["segments"] <= 512
                    assert 3 * p["samples_per_group"] <= p["threads"]
                    assert p["lds_bytes"] <= TILE_MAX_LDS
                    assert p["blocks"] * p["samples_per_group"] >= n
                    assert (p["blocks"] - 1) * p["samples_per_group"] < n
                else:
                    waves = p["threads"] // 64
                    assert p["blocks"] * waves * p["samples_per_group"] >= n
                    assert p["segments"] <= 16


@pytest.mark.parametrize("L", list(range(0, 21)))
def test_backward_plans_fit_the_kernels(L):
    for C in (1, 3, 10, 16, 64):
        MC = (L + 1) ** 2 * C
        for n in NS:
            for shared in (1, 0):
                p = _lib.plan("bwd", n, L, C, shared)
                _check_segments(p, L)
                assert p["threads"] == 64 * p["segments"] <= 512
                assert 3 * p["samples_per_group"] <= p["threads"]
                assert 1 <= p["samples_per_group"] <= 64 // C
                mode = p["tile"]  # backward: spectrum mode (3: persistent kernel)
                assert mode == (0 if not shared else mode) and mode in ((1, 2, 3) if shared else (0,))
                groups = -(-n // p["samples_per_group"])
                slab = -(-MC // 16) * 16
                if mode == 3:
                    # persistent kernel (action_bwd_persist.h): C = 10, l <= 10, from 257
                    # groups; one gradient-tile buffer, 3 blocks per CU, 4 waves; workspace =
                    # one slab per block + the angle-gradient region of the fused path
                    assert C == 10 and 3 <= L <= 10 and groups >= PERSIST_MIN_GROUPS, (L, C, n)
                    assert p["blocks"] == min(groups, PERSIST_BLOCKS) and p["segments"] == 4
                    assert 3 * p["lds_bytes"] <= LDS_PER_CU
                    assert p["aux"] == 4 * p["blocks"] * slab + 4 * 3 * n
                    assert p["aux"] == _lib.load().lv_group_action_bwd_workspace(n, L, C, shared)
                    continue
                assert not (shared and C == 10 and 3 <= L <= 10 and groups >= PERSIST_MIN_GROUPS)
                fallback = mode == 2 or p["lds_bytes"] > BWD_MAX_LDS
                assert p["lds_bytes"] <= (LDS_PER_CU if fallback else BWD_MAX_LDS)
                assert p["blocks"] == min(groups, 1024 if fallback else BWD_MAX_BLOCKS)
                # workspace: the dF slabs, one per block, sized for the chunk-major layout
                # (16-element chunks, action_bwd.h kSlabChunk), then the fused path's
                # angle-gradient region (3 floats per sample)
                assert p["aux"] == (4 * p["blocks"] * slab + 4 * 3 * n if shared else 0)
                assert p["aux"] == _lib.load().lv_group_action_bwd_workspace(n, L, C, shared)


def test_compute_units():
    """The planner sizes the persistent grid by the device's CU count (hipDeviceAttribute-
    MultiprocessorCount); without a device, the MI355X's 256."""
    import torch
    if torch.cuda.is_available():
        assert CUS == torch.cuda.get_device_properties(0).multi_processor_count
    else:
        assert CUS == 256


def test_pinned_plans_of_the_benchmark_configs():
    # config 2 (bench.py): 683 blocks of 6 samples, spectrum in the tile's last slot
    # (6*1210*4 + 16 tile + 6*76*4 trig = 30,880 B -> 5 blocks per CU), write-through
    p = _lib.plan("fwd", 1, 0, F32, 4096, 10, 10)
    assert (p["tile"], p["blocks"], p["lds_bytes"], p["aux"]) == (1, 683, 30880, 1)
    assert _lib.plan("fwd", 1, 0, F32, 65536, 10, 10)["aux"] == 0  # > 32 MB: nt stores
    assert _lib.plan("fwd", 1, 0, F32, 6144, 10, 10)["aux"] == 1   # 29.7 MB: write-through
    assert _lib.plan("fwd", 1, 0, F32, 8192, 10, 10)["aux"] == 0
    # waves per block by sample groups per CU (profiles/r06_ab_nseg_sweep.txt): 7 up to 4
    # groups per CU, 8 up to 16, 4 beyond
    for n, waves in ((4096, 7), (4 * 6 * CUS, 7), (4 * 6 * CUS + 6, 8), (16384, 8),
                     (16 * 6 * CUS, 8), (16 * 6 * CUS + 6, 4), (65536, 4)):
        assert _lib.plan("fwd", 1, 0, F32, n, 10, 10)["segments"] == waves, n
    # config 5: bf16 tile (6*4410*2 + 16, rounded to 16 B) + separate fp32 spectrum copy + trig
    p = _lib.plan("fwd", 1, 0, BF16, 8192, 20, 10)
    assert (p["tile"], p["blocks"], p["lds_bytes"]) == (1, 1366, 52944 + 17640 + 3552)
    # backward at the config-2 size: the persistent kernel (one 6-sample group per block
    # here), 4 waves, LDS small enough for 3 blocks per CU; at one group per CU or less the
    # one-group kernel (profiles/r06_ab_persist_small_batches.txt)
    b = _lib.plan("bwd", 4096, 10, 10, 1)
    assert (b["tile"], b["segments"], b["blocks"], b["samples_per_group"]) == (3, 4, 683, 6)
    assert 3 * b["lds_bytes"] <= 160 * 1024
    assert _lib.plan("bwd", 6 * CUS, 10, 10, 1)["tile"] == 1
    assert _lib.plan("bwd", 6 * CUS + 1, 10, 10, 1)["tile"] == 3
    # config 3's batch (512, one group per CU at most): 8 segments
    assert _lib.plan("bwd", 512, 10, 10, 1)["segments"] == 8
    assert _lib.plan("bwd", 2048, 10, 10, 1)["segments"] == 4
    # every (l, C) has a backward plan; large tiles take the global-spectrum fallback
    assert _lib.plan("bwd", 4096, 20, 64, 1)["tile"] == 2
    assert _lib.plan("bwd", 4096, 20, 13, 1)["tile"] == 1


@pytest.mark.parametrize("args", [
    ("fwd", 1, 0, F32, 16, 21, 10),           # l_max > 20
    ("fwd", 1, 0, F32, 16, 10, 0),            # C < 1
    ("fwd", 1, 0, F32, 16, 10, 65),           # C > 64
    ("fwd", 1, 1210, F32, 16, 10, 10),        # fused path: shared spectrum only
    ("fwd", 0, 1210, BF16, 16, 10, 10),       # bf16 out needs a shared spectrum
    ("fwd", 0, 7, F32, 16, 10, 10),           # bad batch stride
    ("fwd", 1, 0, 5, 16, 10, 10),             # bad dtype
    ("fwd", 1, 0, F32, 0, 10, 10),            # n = 0 has no plan
    ("bwd", 16, 21, 10, 1),
    ("bwd", 0, 10, 10, 1),
])
def test_plan_rejects_bad_arguments(args):
    with pytest.raises(_lib.LieVaeHipError):
        _lib.plan(*args)


_KNOB_SCRIPT = r"""
import json, sys
sys.path.insert(0, sys.argv[1])
from lie_vae import _lib
print(json.dumps([_lib.plan("fwd", 1, 0, _lib.LV_DTYPE_F32, 4096, 10, 10),
                  _lib.plan("bwd", 4096, 10, 10, 1)]))
"""


@pytest.mark.parametrize("lib,honours", [("liblievae_hip.so", False), ("liblievae_hip_ab.so", True)])
def test_product_library_ignores_knobs(lib, honours):
    """The A/B knobs (LV_TILE, LV_TILE_NSEG, LV_BWD_NSEG, LV_BWD_FGLOBAL, ...) are compiled
    into liblievae_hip_ab.so only (-DLV_AB_KNOBS): with them set in the environment the
    product library plans exactly as without, the A/B build changes its plans."""
    import json
    import os
    import subprocess
    import sys
    pkg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lie-vae_amd")
    path = os.path.join(pkg, "lie_vae", lib)

    def run(extra):
        env = {k: v for k, v in os.environ.items() if not k.startswith("LV_")}
        env.update(extra, LIEVAE_HIP_LIB=path)
        r = subprocess.run([sys.executable, "-c", _KNOB_SCRIPT, pkg], env=env, check=True,
                           capture_output=True, text=True, timeout=120)
        return json.loads(r.stdout.strip().splitlines()[-1])

    base = run({})
    knobs = run({"LV_TILE_NSEG": "3", "LV_BWD_NSEG": "2", "LV_BWD_FGLOBAL": "1", "LV_TILE_WT": "0"})
    assert (knobs != base) == honours
    if not honours:
        with open(path, "rb") as f:
            assert b"LV_BWD_NSEG" not in f.read()
