#!/usr/bin/env python3
"""Diagnostic: one-round step-launch time of single-slot vs two-slot (MODE 3) workgroups.
B = n_slots x per_slot envs (all in one round of the 256 CUs): with QCART_DUAL=1 most workgroups straddle
two slots, with QCART_DUAL=0 every slot is padded to whole workgroups. python tools/diag_mixed.py [config]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from deepreinforcementlearningcontrolofquantumcartpoles_amd import config as cfg  # noqa: E402
from deepreinforcementlearningcontrolofquantumcartpoles_amd.core import Stepper  # noqa: E402

conf = cfg.BENCH_CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "metric"]
ph = conf["physics"]
for per_slot in (12, 8, 4):
    B = 21 * per_slot
    acts = torch.arange(B, device="cuda", dtype=torch.int32) % 21
    for dual in ("0", "1"):
        os.environ["QCART_DUAL"] = dual
        st = Stepper(ph, B, 0, seed=1)
        psi = st.new_state()
        if ph.fock:
            st.reset(psi, 1, arg0=16)
        else:
            st.reset(psi, 2, arg0=0.0, arg1=0.0, arg2=1.0)
        n = ph.control_interval
        st.step(psi, acts, n)
        st.set_timing(True)
        for _ in range(3):
            st.step(psi, acts, n)
        tot, launches = st.step_kernel_time()
        st.set_timing(False)
        print(f"per_slot {per_slot:3d} B {B:4d} dual {dual}: {tot / launches:.3f} ms per {n}-step launch", flush=True)

# whole-chip batches: one slot (no padding at all), random slots padded per slot, random slots packed
for B in (4096, 8192):
    for name, acts in (("one slot", torch.full((B,), 7, device="cuda", dtype=torch.int32)),
                       ("random", torch.randint(0, 21, (B,), device="cuda", dtype=torch.int32,
                                                generator=torch.Generator(device="cuda").manual_seed(3)))):
        for dual in ("0", "1"):
            os.environ["QCART_DUAL"] = dual
            st = Stepper(ph, B, 0, seed=1)
            psi = st.new_state()
            if ph.fock:
                st.reset(psi, 1, arg0=16)
            else:
                st.reset(psi, 2, arg0=0.0, arg1=0.0, arg2=1.0)
            n = ph.control_interval
            st.step(psi, acts, n)
            st.set_timing(True)
            for _ in range(3):
                st.step(psi, acts, n)
            tot, launches = st.step_kernel_time()
            st.set_timing(False)
            print(f"B {B} {name:8s} dual {dual}: {tot / launches:.3f} ms per {n}-step launch", flush=True)
