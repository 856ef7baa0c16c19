#!/usr/bin/env python3
"""Summarise the SQ counter passes of tools/gpu_counters.sh (gpurun_out/prof_sq*_<tag>) for the step kernel:
per-launch totals and the per-wave-step derivation (one wave = one env, so per wave-step = per env-step).
Writes profiles/<tag>_sq.txt (readable) and profiles/<tag>_sq.json (bench.py reads the executed-flop count
of a profile whose lib_sha and workload match the run: roofline.binding.executed_*).

  python tools/sq_summary.py TAG [--root gpurun_out] [--no-write]

The workload (envs and physics steps per launch, N, lib_sha) comes from the bench line the profiled run
printed (gpurun_out/prof_sqa_<tag>.log).
"""
import argparse
import collections
import csv
import glob
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def bench_line(root, tag):
    for name in ("sqa", "sqb", "sqc", "sqd", "sqe"):
        f = os.path.join(root, f"prof_{name}_{tag}.log")
        if os.path.exists(f):
            for ln in open(f):
                if ln.startswith("{"):
                    return json.loads(ln)
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--root", default=os.path.join(ROOT, "gpurun_out"))
    ap.add_argument("--no-write", action="store_true")
    a = ap.parse_args()

    tot = collections.defaultdict(float)
    n = collections.Counter()
    kern = set()
    for f in glob.glob(f"{a.root}/prof_sq*_{a.tag}/**/*counter_collection.csv", recursive=True):
        disp = set()
        for r in csv.DictReader(open(f)):
            if "k_step" not in r["Kernel_Name"]:
                continue
            kern.add(r["Kernel_Name"])
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            disp.add((r["Counter_Name"], r["Dispatch_Id"]))
        for c, _ in disp:
            n[c] += 1
    per = {k: tot[k] / max(1, n[k]) for k in tot}
    bl = bench_line(a.root, a.tag)
    lines = []
    for k in sorted(kern):
        lines.append(f"# kernel: {k}")
    if bl:
        lines.append(f"# workload: {bl['config']['workload']}  lib_sha {bl['roofline'].get('lib_sha')}")
    for k in sorted(per):
        lines.append(f"{k:28s} {per[k]:.4g} per launch ({n[k]} launches)")
    der = {}
    if bl:
        envs = bl["config"]["global_batch"] // bl["n_gpus"]
        steps = bl["config"]["physics_steps_per_step"]
        N = bl["config"]["seq_len"]
        ws = envs * steps
        g = per.get
        lines.append(f"# derived (per wave-step = per env-step; {envs} envs x {steps} steps per launch, N = {N}):")
        valu = g("SQ_INSTS_VALU", 0) / ws
        der["valu_insts_per_wave_step"] = valu
        lines.append(f"#   VALU instructions            {valu:.0f}")
        for prec in ("F64", "F32"):
            c = {k: g(f"SQ_INSTS_VALU_{k}_{prec}", 0) / ws for k in ("FMA", "MUL", "ADD")}
            s = sum(c.values())
            if not s:
                continue
            der[f"{prec.lower()}_insts_per_wave_step"] = s
            der[f"{prec.lower()}_fma_mul_add"] = [c["FMA"], c["MUL"], c["ADD"]]
            lines.append(f"#   {prec} VALU (FMA+MUL+ADD)      {s:.0f}  ({s / valu:.0%} of VALU"
                         + ("; a packed v_pk_* counts once" if prec == "F32" else "") + ")")
            lines.append(f"#   FMA / MUL / ADD {prec}          {c['FMA']:.0f} / {c['MUL']:.0f} / {c['ADD']:.0f}")
            if prec == "F64":
                fl = (2 * c["FMA"] + c["MUL"] + c["ADD"]) * 64
                der["f64_flops_per_wave_step_from_insts"] = fl
                lines.append(f"#   FP64 flops from the instruction counts {fl:.0f} per wave-step = {fl / N:.0f} per row")
        for prec in ("FP64", "FP32"):
            k = f"SQ_INSTS_VALU_FLOPS_{prec}"
            if k in per:
                fl = per[k] / ws
                der[f"{prec.lower()}_flops_counter_per_wave_step"] = fl
                # the counter sums each wave instruction's flops of ONE lane (an FMA 2, a v_pk_fma_f32 4): x 64 lanes
                # per wave-step, / N rows
                lines.append(f"#   {k} {fl:.0f} per wave-step (one lane) = {64 * fl / N:.0f} flops per row")
        for k, lab in (("SQ_INSTS_VALU_INT32", "INT32 VALU"), ("SQ_INSTS_VALU_INT64", "INT64 VALU"),
                       ("SQ_INSTS_VALU_CVT", "CVT VALU"), ("SQ_INSTS_VALU_TRANS_F32", "TRANS F32"),
                       ("SQ_INSTS_VALU_TRANS_F64", "TRANS F64"), ("SQ_INSTS_LDS", "LDS instructions"),
                       ("SQ_INSTS_SALU", "SALU instructions"), ("SQ_INSTS_SMEM", "SMEM instructions"),
                       ("SQ_INSTS_VMEM_RD", "VMEM reads"), ("SQ_INSTS_VMEM_WR", "VMEM writes"),
                       ("SQ_INSTS_FLAT", "FLAT (incl. scratch)")):
            if k in per:
                der[k] = per[k] / ws
                lines.append(f"#   {lab:28s} {per[k] / ws:.1f}")
        if "GRBM_GUI_ACTIVE" in per and "SQ_INSTS_VALU" in per:
            clk = per["GRBM_GUI_ACTIVE"] / 8
            der["valu_issue_share"] = per["SQ_INSTS_VALU"] * 4 / (1024 * clk)
            lines.append(f"#   shader clock                 {clk / 1e6:.0f} M cycles per XCD per launch")
            lines.append(f"#   VALU issue share             {der['valu_issue_share']:.2f}"
                         "  (INSTS_VALU x 4 cycles / (1024 SIMDs x clock))")
            f64 = sum(g(f"SQ_INSTS_VALU_{k}_F64", 0) for k in ("FMA", "MUL", "ADD"))
            if f64:
                # a wave64 FP64 FMA occupies the SIMD 4 cycles (78.6 TF = 16 FMA / cycle / SIMD); a 32-bit op 2 cycles
                # when two waves share the SIMD: the share of SIMD cycles the FP64 instructions alone fill
                der["fp64_pipe_share"] = f64 * 4 / (1024 * clk)
                lines.append(f"#   FP64 pipe share              {der['fp64_pipe_share']:.2f}"
                             "  (FP64 FMA/MUL/ADD x 4 cycles / (1024 SIMDs x clock))")
        if "SQ_ACTIVE_INST_VALU" in per and "SQ_WAVE_CYCLES" in per:
            der["active_valu_per_wave_cycle"] = per["SQ_ACTIVE_INST_VALU"] / per["SQ_WAVE_CYCLES"]
            lines.append(f"#   ACTIVE_INST_VALU / WAVE_CYCLES {der['active_valu_per_wave_cycle']:.2f}")
    text = "\n".join(lines)
    print(text)
    if not a.no_write and bl:
        prof = os.path.join(ROOT, "profiles")
        open(os.path.join(prof, f"{a.tag}_sq.txt"), "w").write(
            "# rocprofv3 --pmc SQ counters (tools/gpu_counters.sh, separate passes), per launch of the step kernel\n"
            + text + "\n")
        json.dump({"tag": a.tag, "kernel": sorted(kern), "workload": bl["config"]["workload"],
                   "lib_sha": bl["roofline"].get("lib_sha"), "N": bl["config"]["seq_len"],
                   "envs_per_launch": bl["config"]["global_batch"] // bl["n_gpus"],
                   "steps_per_launch": bl["config"]["physics_steps_per_step"],
                   "per_launch": per, "derived": der}, open(os.path.join(prof, f"{a.tag}_sq.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
