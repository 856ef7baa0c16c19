#!/usr/bin/env python3
"""BASELINE.md §4 run table from the per-config bench lines (profiles/<tag>_<cfg>_bench_line.json) and
rocprofv3 summaries (profiles/<tag>_<cfg>_summary.json) written by tools/run_table.sh + prof_summary.py.
Prints a markdown table and writes profiles/<tag>_run_table.json.  python tools/run_table.py [tag]"""
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROWS = [("C1 HO cooling", "C1"), ("C2 IHO cartpole", "C2"), ("C3 QO cooling", "C3"),
        ("C4 IQO cartpole (per GPU of 8)", "C4"), ("C5 IHO stress (per GPU of 8)", "C5"), ("Metric IHO", "metric")]


def executed_frac(prof, tag, c, bl):
    """Executed FP-VALU fraction: the SQ FLOPS counters of profiles/<tag>_<cfg>_sq.json (tools/sq_summary.py) per
    wave-step x the config's wave-steps per launch / this bench line's k_step time, against the FP64 (FP32 for
    fp32) vector peak. None without the SQ profile."""
    f = os.path.join(prof, f"{tag}_{c}_sq.json")
    if not os.path.exists(f):
        return None
    sq = json.load(open(f))
    # only a profile of this same library build and workload prices this bench line's kernel
    if (sq.get("lib_sha") != bl["roofline"].get("lib_sha")
            or sq.get("workload") != bl["config"].get("workload")):
        return None
    d = sq["derived"]
    fp32 = bl["dtype"] == "f32"
    fl = d.get("fp32_flops_counter_per_wave_step" if fp32 else "fp64_flops_counter_per_wave_step")
    if not fl:
        return None
    ws = bl["config"]["global_batch"] // bl["n_gpus"] * bl["config"]["physics_steps_per_step"]
    peak = 157.3e12 if fp32 else 78.6e12
    return 64.0 * fl * ws / (bl["roofline"]["kernel_ms"] * 1e-3) / peak


def main(tag="r01"):
    prof = os.path.join(ROOT, "profiles")
    out = []
    print("| config | N | B per GPU | dtype | env-steps/s (1 GPU) | k_step ms/launch | HBM-roofline frac "
          "(algorithmic) | FP-VALU frac (nominal) | FP-VALU frac (executed) | rocprof HBM GB/s | "
          "CPU baseline env-steps/s (threads) |")
    print("|---|---|---|---|---|---|---|---|---|---|---|")
    for name, c in ROWS:
        bl = json.loads(open(os.path.join(prof, f"{tag}_{c}_bench_line.json")).read())
        sm = json.load(open(os.path.join(prof, f"{tag}_{c}_summary.json")))
        rf, cpu = bl["roofline"], bl.get("cpu_baseline", {})
        hbm = sm.get("hbm_bytes_per_launch")
        gbs = hbm / (sm["avg_ms"] * 1e-3) / 1e9 if hbm else None
        row = {"config": c, "N": bl["config"]["seq_len"], "batch": bl["config"]["global_batch"], "dtype": bl["dtype"],
               "env_steps_per_s": bl["value"], "kernel_ms": rf["kernel_ms"], "prof_kernel_ms": sm["avg_ms"],
               "hbm_frac": rf["frac"], "valu_frac": (rf["binding"]["frac"] if "binding" in rf else bl["valu"]["frac"]), "rocprof_hbm_gbs": gbs,
               "cpu_env_steps_per_s": cpu.get("value"), "cpu_threads": cpu.get("cores"),
               "cpu_single_core": cpu.get("single_core_value"),
               "valu_frac_executed": executed_frac(prof, tag, c, bl)}
        out.append(row)
        print(f"| {name} | {row['N']} | {row['batch']} | {row['dtype']} | {row['env_steps_per_s']:.3g} | "
              f"{row['kernel_ms']:.3g} | {row['hbm_frac']:.3f} | {row['valu_frac']:.3f} | "
              f"{'%.3f' % row['valu_frac_executed'] if row['valu_frac_executed'] else '-'} | "
              f"{gbs:.0f} | {row['cpu_env_steps_per_s']:.3g} ({row['cpu_threads']}) |")
    json.dump(out, open(os.path.join(prof, f"{tag}_run_table.json"), "w"), indent=1)


if __name__ == "__main__":
    import sys
    main(*sys.argv[1:2])
