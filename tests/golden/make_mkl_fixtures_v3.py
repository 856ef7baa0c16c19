"""Generate tests/golden/mkl_v3.npz: MKL-call-ordered trajectories at the large configuration sizes.

    python tests/golden/make_mkl_fixtures_v3.py      (needs /opt/conda/lib/libmkl_rt.so; this container)

mkl_v1.npz / mkl_v2.npz pin the oracle at the drivers' sizes (IHO 181 / 512, HO 71 / 256, QO 171, IQO 513).
This file extends the pin to the sizes the run table's large configurations step at:

  qo1025   C3's grid: QO x_max 8.5, h 8.5/512 (x_n = 1025, kl = 4 band LU, QO/simulation_quart.cpp:394-432,
           :569-644), dt 1/11520 (the stable dt on that grid), the QO driver's gamma / lambda / mass
  iho1024  IHO N = 1024 (IHO/simulation_i.cpp:432-489), the driver's gamma = 2 pi at dt = 1/5760
  iho2048  C5's IHO N = 2048, gamma = 2 pi at dt = 1/11520

(the reference's README rule — a smaller dt for a larger basis; at the drivers' 1/1440 the top
Fock levels / the fine grid amplify rounding until the run blows up, MKL stepper and oracle alike.)

Each case, through mklref.IhoMkl / GridMkl (every cblas / sparse / LAPACKE call of go_one_step in the
reference's order and descriptors): from a fixed psi0 (|0> for the Fock cases, the drivers' Gaussian packet
on the grid), 1000 steps, one force per control interval decided by a PD rule on the stepper's own <x> history
(then frozen as data), noise = vslNewStream(MT19937, seed) + vdRngGaussian(BOXMULLER) under
MKL_CBWR=COMPATIBLE: psi after 100 / 500 / 1000 steps, every step's q / x_mean / Fail, and for the grid
compute_statistics' 20-moment vector (QO:326-362) of each snapshot. Every array is data (inputs and MKL's
outputs).
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
from math import pi, sqrt

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import mklref as M  # noqa: E402

OUT = os.path.join(HERE, "mkl_v3.npz")
STEPS = 1000
SNAPS = (100, 500, 1000)

CASES = {
    "qo1025": dict(kind="grid", x_max=8.5, h=8.5 / 512, lam=0.04 * pi, mass=1 / pi, gamma=0.01 * pi,
                   dt=1 / 11520, f_max=5.0, ci=160, seed=21025, kp=1.0, kd=1.0, k0=0.2),
    "iho1024": dict(kind="iho", n_max=1023, omega=pi, gamma=2 * pi, dt=1 / 5760, f_max=8.0, ci=80, seed=11024,
                    kp=1.3, kd=0.1),
    "iho2048": dict(kind="iho", n_max=2047, omega=pi, gamma=2 * pi, dt=1 / 11520, f_max=8.0, ci=80, seed=12048,
                    kp=1.3, kd=0.1),
}


def stream_child(out_path: str):
    np.savez(out_path, **{name: M.vsl_gaussian(c["seed"], 2 * STEPS) for name, c in CASES.items()})


def cnr_streams():
    path = "/tmp/_mkl_v3_cnr.npz"
    subprocess.check_call([sys.executable, __file__, "--stream-child", path],
                          env={**os.environ, "MKL_CBWR": "COMPATIBLE"})
    with np.load(path) as z:
        res = {k: z[k] for k in z.files}
    os.unlink(path)
    return res


def psi0_of(c, sim):
    if c["kind"] == "iho":        # the cartpole driver's reset: |0> (IHO/main_parallel.py:231-232)
        psi = np.zeros(c["n_max"] + 1, np.complex128)
        psi[0] = 1.0
        return psi
    x = sim.x                     # Gaussian_packet(1 / k0, 0, 1) (QO/main_parallel.py:177-181)
    return (np.exp(2.j * pi * x * c["k0"]) * np.exp(-x * x / 4.) / sqrt(sqrt(2 * pi))).astype(np.complex128)


def action_of(c, xs):
    """PD rule on <x> at the control step (F = -(kp x + kd dx/dt)) on the 21 force levels; the Fock cases
    clip at +-5 levels (make_mkl_fixtures.py feedback_action)."""
    ci, dt = c["ci"], c["dt"]
    x1 = xs[-1]
    x0 = xs[-1 - ci] if len(xs) > ci else x1
    v = (x1 - x0) / (ci * dt)
    lim = 5 if c["kind"] == "iho" else 10
    a = int(np.clip(np.round(-(c["kp"] * x1 + c["kd"] * v) / (c["f_max"] / 10.)), -lim, lim))
    return 10 + a


def run_case(name, c, r):
    if c["kind"] == "iho":
        sim = M.IhoMkl(c["n_max"], c["omega"])
    else:
        sim = M.GridMkl(c["x_max"], c["h"], c["lam"], c["mass"])
    psi = psi0_of(c, sim)
    out = {f"traj/{name}/psi0": psi.copy()}
    n_int = (STEPS + c["ci"] - 1) // c["ci"]
    acts = np.full(n_int, 10, np.int32)          # no control in the first interval (the drivers' i != 0)
    qs, xs, fs, snaps, moms = [], [], [], [], []
    for k in range(STEPS):
        F = (int(acts[k // c["ci"]]) - 10) * (c["f_max"] / 10.)
        q, xm, f = sim.step(psi, c["dt"], F, c["gamma"], r[k])
        qs.append(q)
        xs.append(xm)
        fs.append(f)
        if k + 1 in SNAPS:
            snaps.append(psi.copy())
            if c["kind"] == "grid":
                moms.append(sim.moments(psi))
        if (k + 1) % c["ci"] == 0 and (k + 1) // c["ci"] < n_int:
            acts[(k + 1) // c["ci"]] = action_of(c, xs)
    out[f"traj/{name}/params"] = np.array(json.dumps(c).encode())
    out[f"traj/{name}/actions"] = acts
    out[f"traj/{name}/noise"] = r
    out[f"traj/{name}/psi"] = np.stack(snaps)
    out[f"traj/{name}/q"] = np.array(qs)
    out[f"traj/{name}/x_mean"] = np.array(xs)
    out[f"traj/{name}/fail"] = np.array(fs, np.int8)
    if moms:
        out[f"traj/{name}/moments"] = np.stack(moms)
    top = np.abs(snaps[-1][-64:]).max()
    print(f"{name}: N={sim.N} |<x>| max {np.abs(xs).max():.3f}, actions {sorted(set(acts.tolist()))}, "
          f"fails {sum(fs)}, max |psi| in the top 64 rows {top:.1e}")
    return out


def main():
    if not M.available():
        sys.exit(f"MKL runtime not found at {M.MKL_PATH}")
    streams = cnr_streams()
    data = {}
    only = [a for a in sys.argv[1:] if a in CASES] or list(CASES)
    for name in only:
        data.update(run_case(name, CASES[name], streams[name].reshape(STEPS, 2)))
    data["meta"] = np.array(json.dumps({
        "mkl": "2021.4.0 (/opt/conda/lib/libmkl_rt.so, conda mkl-2021.4.0-h06a4308_640)",
        "noise": "MKL_CBWR=COMPATIBLE vdRngGaussian(BOXMULLER) of vslNewStream(MT19937, seed)",
        "steps": STEPS, "snapshots": list(SNAPS),
    }).encode())
    np.savez_compressed(OUT, **data)
    print(f"wrote {OUT}: {len(data)} arrays, {os.path.getsize(OUT)} bytes")


if __name__ == "__main__":
    if len(sys.argv) == 3 and sys.argv[1] == "--stream-child":
        stream_child(sys.argv[2])
    else:
        main()
