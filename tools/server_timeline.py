#!/usr/bin/env python3
"""Per-tick timeline of the step server from a rocprofv3 kernel + HIP API trace of the server process
(tools/bench_dropin.py --kinds server --server-prof DIR): for every k_step dispatch, the host's launch call, the
kernel's start and end on the GPU and the first completion poll after it, all on rocprofv3's one clock.
    python3 tools/server_timeline.py DIR [--out FILE]
Prints the median / mean of: launch call -> kernel start (submission latency), kernel duration, kernel end ->
the poll that saw it (completion latency), and the tick period (k_step start to the next k_step start)."""
import argparse
import csv
import glob
import os
import statistics as st


def load(d, what):
    f = glob.glob(os.path.join(d, "**", f"*{what}.csv"), recursive=True)
    if not f:
        raise SystemExit(f"no *{what}.csv under {d}")
    return list(csv.DictReader(open(f[0])))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    ks = load(a.dir, "kernel_trace")
    api = load(a.dir, "hip_api_trace")
    by_corr = {r["Correlation_Id"]: r for r in api}
    polls = sorted(int(r["End_Timestamp"]) for r in api if r["Function"] in ("hipEventQuery", "hipStreamSynchronize"))
    steps = sorted((r for r in ks if "k_step" in r["Kernel_Name"]), key=lambda r: int(r["Start_Timestamp"]))
    import bisect
    sub, dur, done, period = [], [], [], []
    prev = None
    for r in steps:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        c = by_corr.get(r["Correlation_Id"])
        if c is not None:
            sub.append((s - int(c["End_Timestamp"])) / 1e3)
        dur.append((e - s) / 1e3)
        i = bisect.bisect_left(polls, e)
        if i < len(polls):
            done.append((polls[i] - e) / 1e3)
        if prev is not None:
            period.append((s - prev) / 1e3)
        prev = s
    names = {}
    for r in ks:
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        names.setdefault(n, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    lines = [f"# tools/server_timeline.py {a.dir}: {len(steps)} k_step dispatches (us)"]
    for lab, v in (("launch call end -> kernel start", sub), ("k_step duration", dur),
                   ("kernel end -> completion poll", done), ("tick period (k_step to k_step)", period)):
        if v:
            lines.append(f"{lab:34s} median {st.median(v):8.2f}  mean {st.mean(v):8.2f}  n {len(v)}")
    for n, v in sorted(names.items(), key=lambda kv: -sum(kv[1])):
        lines.append(f"kernel {n[:60]:60s} calls {len(v):7d} mean {st.mean(v):8.2f} us")
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        open(a.out, "w").write(txt + "\n")


if __name__ == "__main__":
    main()
