"""Per-kernel table of a steady-state training profile (tools/gpu_train_prof.sh).

  python tools/train_kernel_table.py <kernel_stats.csv> <steps> [<pmc dir>] > table.txt

<steps>: training steps the profiled process ran (warm-up + FLOP-count step + timed), so
each kernel's time per step = total / steps.  With a PMC directory (one rocprofv3 --pmc
pass holding SQ_VALU_MFMA_BUSY_CYCLES and GRBM_GUI_ACTIVE) each kernel also gets its
MFMA utilisation: MFMA-busy SIMD-cycles / (1024 SIMDs x the dispatch's cycles), the
dispatch's cycles = GRBM_GUI_ACTIVE / 8 XCDs (MI355X_MICROARCH.md: SQ_VALU_MFMA_BUSY_CYCLES
counts 32 cycles per 32x32x16 bf16 MFMA; GRBM_GUI_ACTIVE sums the 8 XCDs).
"""
import csv
import glob
import sys
from collections import defaultdict

stats, steps = sys.argv[1], float(sys.argv[2])
pmc = sys.argv[3] if len(sys.argv) > 3 else None
rows = list(csv.DictReader(open(stats)))
total = sum(float(r["TotalDurationNs"]) for r in rows)
mfma = {}
if pmc:
    acc = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(f"{pmc}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            acc[r["Kernel_Name"]][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, c in acc.items():
        cyc = c.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        if cyc > 0:
            mfma[k] = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (1024.0 * cyc)
print(f"# {stats}: {total / 1e6:.2f} ms of kernels over {steps:g} steps = "
      f"{total / 1e6 / steps:.3f} ms/step")
print(f"{'ms/step':>8} {'%':>6} {'calls/step':>10} {'avg us':>9} {'MFMA util':>9}  kernel")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    t = float(r["TotalDurationNs"])
    name = r["Name"]
    u = next((v for k, v in mfma.items() if k.startswith(name[:60])), None)
    us = f"{100 * u:8.1f}%" if u is not None else f"{'-':>9}"
    print(f"{t / 1e6 / steps:8.3f} {100 * t / total:6.2f} {float(r['Calls']) / steps:10.2f} "
          f"{float(r['AverageNs']) / 1e3:9.2f} {us}  {name[:110]}")
