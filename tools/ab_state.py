#!/usr/bin/env python3
"""Diagnostic: run a fixed IHO workload (Philox noise, random actions) with the library QCART_LIB points
at and save the final states, so two builds can be compared bitwise:
  QCART_LIB=... python tools/ab_state.py out.npy [n_max] [batch] [steps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from deepreinforcementlearningcontrolofquantumcartpoles_amd import config as cfg  # noqa: E402
from deepreinforcementlearningcontrolofquantumcartpoles_amd.core import Stepper  # noqa: E402


def main():
    out = sys.argv[1]
    n_max = int(sys.argv[2]) if len(sys.argv) > 2 else 511
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 160
    fam = int(os.environ.get("AB_FAMILY", cfg.IHO))
    ph = cfg.DEFAULTS[fam].with_(n_max=n_max)
    st = Stepper(ph, B, 0, seed=11)
    psi = st.new_state()
    st.reset(psi, 1, arg0=16)
    g = torch.Generator(device="cuda").manual_seed(4)
    res = []
    for c in range(steps // 80):
        acts = torch.randint(0, 21, (B,), generator=g, device="cuda", dtype=torch.int32)
        o = st.step(psi, acts, 80, want_fail=True)
        res.append(o["fail_step"].cpu().numpy())
    np.savez(out, psi=psi.cpu().numpy(), fail=np.stack(res))
    print("saved", out, flush=True)


if __name__ == "__main__":
    main()
