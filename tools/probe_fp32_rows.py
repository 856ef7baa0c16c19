#!/usr/bin/env python3
"""Row-steps per second of the fp32 IHO step kernels at N = 1024 (R = 16: two waves per SIMD) and N = 2048 (R = 32,
C5: one wave per SIMD), random actions, 80-step launches: how much a wave pair per env (R = 16 per wave, the
DESIGN §10 plan for C5) could gain before its exchange cost.   python3 tools/probe_fp32_rows.py [--batch 32768]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deepreinforcementlearningcontrolofquantumcartpoles_amd import config as cfg  # noqa: E402
from deepreinforcementlearningcontrolofquantumcartpoles_amd.core import Stepper  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32768)
    ap.add_argument("--launches", type=int, default=3)
    a = ap.parse_args()
    out = {}
    for n_max in (1023, 2047):
        ph = cfg.DEFAULTS[cfg.IHO].with_(n_max=n_max, precision=1)
        st = Stepper(ph, a.batch, 0, seed=1)
        psi = st.new_state()
        st.reset(psi, 1, arg0=16)
        acts = torch.randint(0, 21, (a.batch,), dtype=torch.int32, device="cuda")
        st.step(psi, acts, 80)                    # warm-up
        st.sync()
        st.set_timing(True)
        st.step_kernel_time()
        for _ in range(a.launches):
            st.step(psi, acts, 80)
        ms, n = st.step_kernel_time()
        per = ms / n
        rows = (n_max + 1) * a.batch * 80
        out[n_max + 1] = {"ms_per_launch": per, "row_steps_per_s": rows / (per * 1e-3)}
        st.close()
    out["ratio_row_rate_1024_over_2048"] = out[1024]["row_steps_per_s"] / out[2048]["row_steps_per_s"]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
