#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel-trace/stats run and the FETCH_SIZE / WRITE_SIZE PMC passes into
profiles/<tag>_summary.json (+ copies of the stats CSVs) for the judge and for bench.py's
roofline.traffic field.

HBM bytes per launch, corrected as MI355X_MICROARCH.md §HBM prescribes: FETCH_SIZE (KiB) counts
half of the bytes of wide coalesced 16-B/lane reads on gfx950 -> x2; WRITE_SIZE (KiB) is exact for
16-B/lane stores.
"""
import csv
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(tag, kernel="k_step"):
    out = os.path.join(ROOT, "gpurun_out")
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = os.path.join(out, f"prof_kt_{tag}", "run_kernel_stats.csv")
    rows = list(csv.DictReader(open(stats)))
    shutil.copy(stats, os.path.join(prof, f"{tag}_kernel_stats.csv"))
    k = [r for r in rows if kernel in r["Name"]][0]
    res = {"tag": tag, "kernel": k["Name"], "calls": int(k["Calls"]), "avg_ms": float(k["AverageNs"]) / 1e6,
           "min_ms": float(k["MinNs"]) / 1e6, "max_ms": float(k["MaxNs"]) / 1e6}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        f = os.path.join(out, f"prof_pmc_{c}_{tag}", "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if kernel in r["Kernel_Name"]]
        shutil.copy(f, os.path.join(prof, f"{tag}_pmc_{c}.csv"))
        res[c + "_KiB_median"] = statistics.median(vals)
    if "FETCH_SIZE_KiB_median" in res and "WRITE_SIZE_KiB_median" in res:
        rd = 2.0 * res["FETCH_SIZE_KiB_median"] * 1024
        wr = res["WRITE_SIZE_KiB_median"] * 1024
        res["hbm_read_bytes_per_launch"] = rd
        res["hbm_write_bytes_per_launch"] = wr
        res["hbm_bytes_per_launch"] = rd + wr
    log = os.path.join(out, f"prof_kt_{tag}.log")
    if os.path.exists(log):
        for line in open(log):
            if line.startswith("{"):
                res["bench_line"] = json.loads(line)
    json.dump(res, open(os.path.join(prof, f"{tag}_summary.json"), "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "bench_line"}, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
