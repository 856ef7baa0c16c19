#!/usr/bin/env python3
"""Diagnostic: C2-size (B = 4096, IHO N = 512) step-launch time by action layout."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from deepreinforcementlearningcontrolofquantumcartpoles_amd import config as cfg  # noqa: E402
from deepreinforcementlearningcontrolofquantumcartpoles_amd.core import Stepper  # noqa: E402

ph = cfg.BENCH_CONFIGS["C2"]["physics"]
B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
g = torch.Generator(device="cuda").manual_seed(3)
seq = sys.argv[2] if len(sys.argv) > 2 else "01"
cases = {f"slot {s}": torch.full((B,), s, device="cuda", dtype=torch.int32) for s in (0, 7, 10, 20)}
cases["slots 0/20"] = (torch.arange(B, device="cuda", dtype=torch.int32) % 2) * 20
cases["random"] = torch.randint(0, 21, (B,), device="cuda", dtype=torch.int32, generator=g)
cases["random 8..12"] = torch.randint(8, 13, (B,), device="cuda", dtype=torch.int32, generator=g)
if "pre" in sys.argv:   # a small two-slot launch first (as tools/diag_mixed.py does)
    os.environ["QCART_DUAL"] = "1"
    st0 = Stepper(ph, 252, 0, seed=1)
    p0 = st0.new_state()
    st0.reset(p0, 1, arg0=16)
    st0.step(p0, torch.arange(252, device="cuda", dtype=torch.int32) % 21, 80)
    torch.cuda.synchronize()
    del st0, p0
if "small" in sys.argv:   # tools/diag_mixed.py's one-round section first
    for per_slot in (12, 8, 4):
        Bs = 21 * per_slot
        a_s = torch.arange(Bs, device="cuda", dtype=torch.int32) % 21
        for dual in ("0", "1"):
            os.environ["QCART_DUAL"] = dual
            st = Stepper(ph, Bs, 0, seed=1)
            p0 = st.new_state()
            st.reset(p0, 1, arg0=16)
            for _ in range(4):
                st.step(p0, a_s, 80)
            torch.cuda.synchronize()
if "slot7" in sys.argv:
    cases = {"slot 7": cases["slot 7"]}
for name, acts in cases.items():
    for dual in seq:
        os.environ["QCART_DUAL"] = dual
        st = Stepper(ph, B, 0, seed=1)
        psi = st.new_state()
        st.reset(psi, 1, arg0=16)
        st.step(psi, acts, 80)
        st.set_timing(True)
        for _ in range(3):
            st.step(psi, acts, 80)
        tot, n = st.step_kernel_time()
        st.set_timing(False)
        order, mixed = st.group_layout()
        busy = int((order >= 0).any(1).sum()) + int((mixed >= 0).any(1).sum())
        print(f"{name:14s} dual {dual}: {tot / n:.3f} ms  ({busy} workgroups)", flush=True)
print("scan levels per slot:", [st.scan_levels(a) for a in range(21)])
