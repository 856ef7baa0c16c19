#!/usr/bin/env python3
"""Break the end-to-end actor loop (tools/bench_loop.py) down by kernel and host gap: one rocprofv3 run with the
kernel trace and the roctx marker trace; the kernels whose dispatch lies inside bench_loop's 'timed' range are
summed per name and per control step, and the GPU-idle time is the range's wall time minus the union of the
kernel intervals (host work, syncs and launch latency the GPU waits on).
The parent never touches the GPU (rocprofv3 runs bench_loop as its own child).
python3 tools/loop_breakdown.py [--batch 65536] [--steps 20] [--out profiles/<tag>_loop_breakdown.txt]"""
import argparse
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    n = name.replace("(anonymous namespace)::", "").split("(")[0]
    for p in ("void ", "qcart::"):
        n = n.replace(p, "")
    if "at::native" in n or "at::" in n:
        n = "torch:" + n.split("<")[0].split("::")[-1]
    return n[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--input", default="xp")
    ap.add_argument("--reset", default="deferred", choices=("immediate", "deferred"))
    ap.add_argument("--out", default="")
    ap.add_argument("--dir", default=os.path.join(ROOT, "gpurun_out", "loop_bd"))
    a = ap.parse_args()
    env = dict(os.environ, TMPDIR="/tmp")
    cmd = ["rocprofv3", "--kernel-trace", "--marker-trace", "--output-format", "csv", "-d", a.dir, "-o", "run", "--",
           sys.executable, os.path.join(ROOT, "tools", "bench_loop.py"), "--batch", str(a.batch), "--steps",
           str(a.steps), "--input", a.input, "--reset", a.reset, "--marker"]
    r = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True, timeout=900)
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not line:
        sys.exit(f"bench_loop under rocprofv3 failed rc={r.returncode}\n{r.stdout[-2000:]}\n{r.stderr[-3000:]}")
    res = json.loads(line[-1])
    kt = glob.glob(os.path.join(a.dir, "**", "run_kernel_trace.csv"), recursive=True)[0]
    mk = glob.glob(os.path.join(a.dir, "**", "run_marker_api_trace.csv"), recursive=True)[0]
    t0 = t1 = None
    for row in csv.DictReader(open(mk)):
        if "timed" in row.get("Function", "") + row.get("Kind", "") + row.get("Message", "") + str(row):
            t0, t1 = int(row["Start_Timestamp"]), int(row["End_Timestamp"])
    if t0 is None:
        sys.exit("no 'timed' marker range in " + mk)
    ks = []
    for row in csv.DictReader(open(kt)):
        s, e = int(row["Start_Timestamp"]), int(row["End_Timestamp"])
        if s >= t0 and e <= t1:
            ks.append((s, e, short(row["Kernel_Name"])))
    ks.sort()
    K = a.steps
    per = {}
    for s, e, n in ks:
        c = per.setdefault(n, [0, 0.0])
        c[0] += 1
        c[1] += (e - s) / 1e6
    busy, cur_s, cur_e = 0.0, None, None   # union of the kernel intervals
    for s, e, _ in ks:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += (cur_e - cur_s) / 1e6
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += (cur_e - cur_s) / 1e6
    wall = (t1 - t0) / 1e6
    lines = [f"# tools/loop_breakdown.py: bench_loop --batch {a.batch} --steps {K} --input {a.input} --reset {a.reset} under rocprofv3 "
             f"(kernel + marker trace), the 'timed' range only",
             f"# bench_loop: {res['ms_per_control_step']:.2f} ms per control step (its own clock, profiled run), "
             f"done fraction per control step {res.get('done_fraction_per_control_step', float('nan')):.4f}",
             f"timed range {wall / K:8.3f} ms per control step; GPU busy (union of kernels) {busy / K:8.3f}; "
             f"GPU idle {(wall - busy) / K:8.3f}",
             f"{'kernel':60s} {'calls/step':>10s} {'ms/step':>9s}"]
    for n, (c, ms) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        lines.append(f"{n:60s} {c / K:10.2f} {ms / K:9.3f}")
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        open(a.out, "w").write(txt + "\n")


if __name__ == "__main__":
    main()
