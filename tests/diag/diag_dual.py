"""Diagnostic (GPU): two-slot remainder workgroups vs per-slot padded ones — per-field differences and
each side against the oracle. python tests/diag/diag_dual.py [case]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from deepreinforcementlearningcontrolofquantumcartpoles_amd import config as cfg  # noqa: E402
from deepreinforcementlearningcontrolofquantumcartpoles_amd.core import Stepper  # noqa: E402
from oracle import oracle as O  # noqa: E402

case = sys.argv[1] if len(sys.argv) > 1 else "iho512"
philox = len(sys.argv) > 2 and sys.argv[2] == "philox"
ph = {"iho512": cfg.DEFAULTS[cfg.IHO].with_(n_max=511), "ho256": cfg.DEFAULTS[cfg.HO].with_(n_max=255),
      "iqo513": cfg.DEFAULTS[cfg.IQO].with_(x_max=12.8), "qo171": cfg.DEFAULTS[cfg.QO]}[case]
B = 203
rng = np.random.default_rng(5)
counts = {0: 3, 2: 8, 3: 1, 5: 40, 7: 9, 10: 61, 11: 7, 13: 17, 17: 33, 20: 24}
acts = rng.permutation(np.concatenate([np.full(c, s, np.int32) for s, c in counts.items()]))
budget = np.full(B, 30, np.int32)
budget[rng.choice(B, 12, replace=False)] = 0
budget[rng.choice(B, 5, replace=False)] = 17
res = {}
for dual in ("1", "0"):
    os.environ["QCART_DUAL"] = dual
    st = Stepper(ph, B, 0, seed=21)
    psi = st.new_state()
    if ph.fock:
        st.reset(psi, 1, arg0=16)
    else:
        st.reset(psi, 2, arg0=0.0, arg1=0.0, arg2=1.0)
    psi0 = psi.cpu().numpy().copy()
    nz = torch.randn((30, B, 2), dtype=torch.float64, device="cuda", generator=torch.Generator("cuda").manual_seed(3))
    out = st.step(psi, torch.from_numpy(acts).cuda(), 30, env_steps=torch.from_numpy(budget).cuda(), want_q=True,
                  noise=None if philox else nz)
    torch.cuda.synchronize()
    res[dual] = (psi.cpu().numpy(), out["q"].cpu().numpy(), out["fail_step"].cpu().numpy())
d = np.abs(res["1"][0] - res["0"][0]).max(axis=1)
bad = np.nonzero(d)[0]
print("psi max diff", d.max(), "envs differing", len(bad), "slots", sorted(set(acts[bad].tolist())))
osys = O.OracleSystem(ph.family, n_max=ph.n_max, omega=ph.omega, x_max=ph.x_max, grid_size=ph.grid_size,
                      lambda_=ph.lambda_, mass=ph.mass)
nzc = nz.cpu().numpy()
for e in bad[:6]:
    ref = psi0[e:e + 1].copy()
    n = int(budget[e])
    if n and philox:
        osys.run_batch(ref, acts[e:e + 1], ph.f_max, n, ph.dt, ph.gamma, seed=21, env_offset=int(e), n_threads=1)
    elif n:
        osys.run_batch(ref, acts[e:e + 1], ph.f_max, n, ph.dt, ph.gamma, noise=nzc[:n, e:e + 1].copy(), n_threads=1)
    print(f"env {e} slot {acts[e]} budget {n}: dual-ref {np.abs(res['1'][0][e] - ref[0]).max():.3e} "
          f"padded-ref {np.abs(res['0'][0][e] - ref[0]).max():.3e} dual-padded {d[e]:.3e}")
