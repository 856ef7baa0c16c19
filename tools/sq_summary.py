#!/usr/bin/env python3
"""Print per-launch SQ counter totals of the step kernel from gpurun_out/prof_sq*_<tag>."""
import collections
import csv
import glob
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
tot = collections.defaultdict(float)
n = collections.Counter()
for f in glob.glob(f"gpurun_out/prof_sq*_{tag}/**/*counter_collection.csv", recursive=True):
    disp = set()
    for r in csv.DictReader(open(f)):
        if "k_step" not in r["Kernel_Name"]:
            continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
        disp.add((r["Counter_Name"], r["Dispatch_Id"]))
    for c, _ in disp:
        n[c] += 1
for k in sorted(tot):
    print(f"{k:28s} {tot[k] / max(1, n[k]):.4g} per launch ({n[k]} launches)")
