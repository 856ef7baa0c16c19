"""Generate tests/golden/golden_v1.npz from the CPU restatement (oracle/).

The reference ships no golden vectors and could not be run here, so these fixtures
freeze the oracle's outputs: they pin the oracle against silent drift (tests/test_golden.py, CPU) and
give the HIP path a fixed target (tests/test_gpu_golden.py). Regenerate only on a deliberate
change of the restated algorithm:  python tests/golden/make_golden.py

Each case: 4 envs, 200 physics steps in 5 control intervals of 40 with fixed per-interval actions,
in-kernel-style Philox noise (seed 11, env ids 0..3), no boundary Fail allowed.
"""
from __future__ import annotations

import os
import sys
from math import pi, sqrt

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from deepreinforcementlearningcontrolofquantumcartpoles_amd import config as cfg  # noqa: E402
from oracle import oracle as O  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden_v1.npz")
SEED, B, CHUNK, N_CHUNK = 11, 4, 40, 5

CASES = {
    "iho64": cfg.DEFAULTS[cfg.IHO].with_(n_max=63, gamma=0.5 * pi),
    "iho64_exact": cfg.DEFAULTS[cfg.IHO].with_(n_max=63, gamma=0.5 * pi, a_mode=1),
    "ho71": cfg.DEFAULTS[cfg.HO],
    "qo171": cfg.DEFAULTS[cfg.QO],
    "iqo257": cfg.DEFAULTS[cfg.IQO].with_(x_max=6.4),
}


def osys(ph):
    return O.OracleSystem(ph.family, n_max=ph.n_max, omega=ph.omega, x_max=ph.x_max,
                          grid_size=ph.grid_size, lambda_=ph.lambda_, mass=ph.mass,
                          moment_order=ph.moment_order, a_mode=ph.a_mode)


def initial(s, ph):
    if ph.fock:
        return np.stack([s.fock_random_state(5, e, 8) for e in range(B)])
    out = []
    for e in range(B):
        psi = s.gaussian_packet(0.1 * e - 0.15, 0.2 * e - 0.3, 0.8 + 0.1 * e)
        out.append(psi / (np.linalg.norm(psi) * sqrt(ph.grid_size)))
    return np.stack(out)


def make_case(name, ph):
    s = osys(ph)
    psi0 = initial(s, ph)
    half = ph.n_actions // 2
    acts = (half + ((np.arange(N_CHUNK)[:, None] * 3 + np.arange(B)[None, :] * 2) % 5) - 2).astype(np.int32)
    psi = psi0.copy()
    qs, xs = [], []
    for c in range(N_CHUNK):
        fail, q, xm = s.run_batch(psi, acts[c], ph.f_max, CHUNK, ph.dt, ph.gamma, seed=SEED,
                                  step0=c * CHUNK, want_q=True, n_threads=1)
        assert not fail.any(), (name, c, fail)
        qs.append(q)
        xs.append(xm)
    obs = np.stack([s.moments(p) for p in psi])
    return {
        f"{name}/params": np.array([ph.family, ph.n_max, ph.omega, ph.x_max, ph.grid_size, ph.lambda_,
                                    ph.mass, ph.moment_order, ph.a_mode, ph.gamma, ph.dt, ph.f_max]),
        f"{name}/psi0": psi0,
        f"{name}/actions": acts,
        f"{name}/psi": psi,
        f"{name}/q": np.concatenate(qs),
        f"{name}/x_mean": np.concatenate(xs),
        f"{name}/obs": obs,
        f"{name}/x_expectation": np.array([s.x_expectation(p) for p in psi]),
        f"{name}/energy": np.array([s.energy(p) if not ph.fock else np.nan for p in psi]),
        f"{name}/phonon": np.array([s.phonon(p) if ph.fock else np.nan for p in psi]),
    }


def main():
    data = {}
    for name, ph in CASES.items():
        data.update(make_case(name, ph))
    ctrs = np.array([[0, 0, 0, 0], [0xFFFFFFFF] * 4, [0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344],
                     [5, 0, 3, 0], [7, 0, 1, 1]], dtype=np.uint32)
    keys = np.array([[0, 0], [0xFFFFFFFF] * 2, [0xA4093822, 0x299F31D0], [11, 0], [11, 0]], dtype=np.uint32)
    data["philox/ctr"] = ctrs
    data["philox/key"] = keys
    data["philox/out"] = np.stack([O.philox(c, k) for c, k in zip(ctrs, keys)])
    data["normals/ids"] = np.array([[11, e, k] for e in range(3) for k in (0, 1, 63, 64, 1000)], dtype=np.int64)
    data["normals/out"] = np.stack([O.normals(int(a), int(b), int(c)) for a, b, c in data["normals/ids"]])
    np.savez_compressed(OUT, **data)
    print(f"wrote {OUT}: {len(data)} arrays, {os.path.getsize(OUT)} bytes")


if __name__ == "__main__":
    main()
