#!/usr/bin/env python3
"""Per-kernel PMC totals (averaged over dispatches) from gpurun_out/prof_<pass>_<tag> dirs:
python3 tools/pmc_table.py <tag> <pass> [<pass> ...]"""
import collections
import csv
import glob
import sys

tag, passes = sys.argv[1], sys.argv[2:]
tot = collections.defaultdict(float)
disp = collections.defaultdict(set)
for p in passes:
    for f in glob.glob(f"gpurun_out/prof_{p}_{tag}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:48]
            tot[(k, r["Counter_Name"])] += float(r["Counter_Value"])
            disp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
for k in sorted({k for k, _ in tot}):
    print(k)
    for (kk, c), v in sorted(tot.items()):
        if kk == k:
            print(f"   {c:34s} {v / len(disp[(kk, c)]):.4g}")
