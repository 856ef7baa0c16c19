#!/usr/bin/env python3
"""Diagnostic: k_step launch time at the metric workload under different action layouts and
physics modes (random / uniform / sorted-by-action; reference vs exact term7). Not the bench.
usage: python tools/diag_actions.py [--batch B] [--reps K]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from deepreinforcementlearningcontrolofquantumcartpoles_amd import config as cfg  # noqa: E402
from deepreinforcementlearningcontrolofquantumcartpoles_amd.core import Stepper  # noqa: E402


def timeit(st, psi, acts, n, reps):
    st.step(psi, acts, n)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s = torch.cuda.current_stream()
    e0.record(s)
    for _ in range(reps):
        st.step(psi, acts, n)
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--config", default="metric")
    ap.add_argument("--n-max", type=int, default=0)
    ap.add_argument("--only", default="", help="comma list of layouts (random,uniform,sorted)")
    args = ap.parse_args()
    B = args.batch
    base = cfg.BENCH_CONFIGS[args.config]["physics"]
    if args.n_max:
        base = base.with_(n_max=args.n_max)
    for mode_name, ph in (("ref", base), ("exact", base.with_(a_mode=1))):
        st = Stepper(ph, B, 0, seed=1)
        psi = st.new_state()
        st.reset(psi, 1, arg0=16) if ph.fock else st.reset(psi, 2, arg0=0.0, arg1=0.0, arg2=1.0)
        g = torch.Generator(device="cuda").manual_seed(3)
        rnd = torch.randint(0, ph.n_actions, (B,), generator=g, device="cuda", dtype=torch.int32)
        layouts = {"random": rnd, "uniform": torch.full_like(rnd, ph.n_actions // 2),
                   "sorted": torch.sort(rnd).values}
        n = ph.control_interval
        for name, acts in layouts.items():
            if args.only and name not in args.only.split(","):
                continue
            ms = timeit(st, psi, acts, n, args.reps)
            print(f"N={ph.dim:5d} {mode_name:6s} {name:8s} {ms:8.2f} ms/launch  {B * n / ms * 1e3:.4g} env-steps/s"
                  f"  {B * n * ph.dim / ms * 1e3:.4g} row-steps/s", flush=True)


if __name__ == "__main__":
    main()
