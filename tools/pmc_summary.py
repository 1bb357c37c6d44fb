"""Summarise rocprofv3 --pmc CSVs: mean counter value per dispatch of each kernel."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
match = sys.argv[2] if len(sys.argv) > 2 else "action"
acc = defaultdict(list)
for f in sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)):
    for row in csv.DictReader(open(f)):
        if match not in row["Kernel_Name"]:
            continue
        acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, v in acc.items():
    print(f"{k:28s} {sum(v) / len(v):16.1f}   (n={len(v)})")
