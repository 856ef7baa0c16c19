#!/usr/bin/env python3
"""The metric's step kernel body inside the one-launch two-slot kernel (k_step DUAL) against the plain single-slot
kernel on a batch that needs no two-slot workgroup (every force slot holds a multiple of 8 envs, so both layouts run
the same 8 192 workgroups): run once with QCART_DUAL=1 (default) and once with QCART_DUAL=0, compare kernel_ms.
python3 tools/probe_dual_body.py [--launches 5]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from deepreinforcementlearningcontrolofquantumcartpoles_amd import config as cfg  # noqa: E402
from deepreinforcementlearningcontrolofquantumcartpoles_amd.core import Stepper  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=5)
    a = ap.parse_args()
    conf = cfg.BENCH_CONFIGS["metric"]
    ph, B = conf["physics"], conf["batch"]
    st = Stepper(ph, B, 0, seed=42)
    psi = st.new_state()
    st.reset(psi, 1, arg0=16)
    e = torch.arange(B, device="cuda", dtype=torch.int64)
    acts = ((e // 8) % ph.n_actions).to(torch.int32)     # 8-env runs per slot: no two-slot workgroup
    st.step(psi, acts, 80)
    st.sync()
    st.set_timing(True)
    st.step_kernel_time()
    for _ in range(a.launches):
        st.step(psi, acts, 80, want_obs=True)
    ms, n = st.step_kernel_time()
    single, mixed = st.group_layout()
    print(json.dumps({"dual_env": os.environ.get("QCART_DUAL", "1"), "kernel_ms": ms / n, "launches": n,
                      "two_slot_workgroups": int(len(mixed))}))


if __name__ == "__main__":
    main()
