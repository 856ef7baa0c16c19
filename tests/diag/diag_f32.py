#!/usr/bin/env python3
"""Diagnostic: fp32 path (config C5) vs the fp64 oracle, and its launch time at the C5 per-GPU batch."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from deepreinforcementlearningcontrolofquantumcartpoles_amd import config as cfg  # noqa: E402
from deepreinforcementlearningcontrolofquantumcartpoles_amd.core import Stepper  # noqa: E402
from oracle import oracle as O  # noqa: E402


def main():
    for n_max in (511, 2047):
        ph = cfg.DEFAULTS[cfg.IHO].with_(n_max=n_max, precision=1, gamma=0.5 * np.pi)
        B = 4
        s = O.OracleSystem(ph.family, n_max=ph.n_max)
        psi0 = np.zeros((B, ph.dim), np.complex128)
        psi0[:, 0] = 1.0
        st = Stepper(ph, B, 0, seed=1)
        g = torch.from_numpy(psi0.astype(np.complex64)).cuda()
        ref = psi0.copy()
        rng = np.random.default_rng(0)
        for c in range(5):
            acts = rng.integers(8, 13, B).astype(np.int32)
            nz = rng.standard_normal((40, B, 2))
            s.run_batch(ref, acts, ph.f_max, 40, ph.dt, ph.gamma, noise=nz, n_threads=4)
            st.step(g, torch.from_numpy(acts).cuda(), 40, noise=torch.from_numpy(nz).cuda())
            err = np.linalg.norm(g.cpu().numpy().astype(np.complex128) - ref, axis=1)
            print(f"N={ph.dim} step {40 * (c + 1)}: |psi32 - psi64| = {err.max():.3e}", flush=True)
    ph = cfg.BENCH_CONFIGS["C5"]["physics"]
    B = cfg.BENCH_CONFIGS["C5"]["batch"] // 8
    st = Stepper(ph, B, 0, seed=1)
    psi = st.new_state()
    st.reset(psi, 1, arg0=16)
    acts = torch.randint(0, 21, (B,), device="cuda", dtype=torch.int32)
    st.step(psi, acts, 80)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        st.step(psi, acts, 80)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 3
    norms = (psi.abs() ** 2).sum(1)
    print(f"C5 fp32 N={ph.dim} B={B}: {ms:.2f} ms / 80 steps, {B * 80 / ms * 1e3:.4g} env-steps/s, "
          f"{16 * ph.dim * B * 80 / ms / 1e6:.1f} GB/s algorithmic, |norm-1| max {float((norms - 1).abs().max()):.2e}")


if __name__ == "__main__":
    main()
