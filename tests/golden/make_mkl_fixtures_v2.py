"""Generate tests/golden/mkl_v2.npz: MKL-call-ordered trajectories of the harmonic and grid families.

    python tests/golden/make_mkl_fixtures_v2.py      (needs /opt/conda/lib/libmkl_rt.so; this container)

mkl_v1.npz pins the IHO go_one_step end to end; this file does the same for the other three reference
modules, through the steppers of mklref.py that restate their MKL call sequences:

  traj/<case>   mklref.HoMkl (HO/simulation.cpp) or mklref.GridMkl (QO/simulation_quart.cpp, also the
                inverted quartic's module) from a fixed psi0, 1000 steps, one force per control interval
                (decided by a PD rule on the stepper's own <x> history, then frozen as data), noise = the
                reference's stream vslNewStream(MT19937, seed) + vdRngGaussian(BOXMULLER) under
                MKL_CBWR=COMPATIBLE: psi after 100 / 500 / 1000 steps, every step's q / x_mean / Fail, and
                for the grid families compute_statistics' 20-moment vector (QO:326-362) of each snapshot.

zero/*        the reference stream with planted zero words (vslSaveStreamM / vslLoadStreamM): the state (mt[624]
              + read index) and MKL's next 8 BOXMULLER normals — MKL's answer for u1 = 0.

Cases: ho71 (HO driver n_max 70), ho256 (C1's N = 256), qo171 (QO driver grid x_max 8.5, h 0.1),
iqo513 (C4's x_max 12.8, h 0.05, dt 1/2880). Every array is data (inputs and MKL's outputs).
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

OUT = os.path.join(HERE, "mkl_v2.npz")
STEPS = 1000
SNAPS = (100, 500, 1000)

# physics per the drivers' arguments (config.DEFAULTS): gamma, dt, F_max, control interval
CASES = {
    "ho71": dict(kind="ho", n_max=70, omega=pi, gamma=pi, dt=1 / 1440, f_max=5.0, ci=80, seed=1071,
                 kp=0.0, kd=1.5),
    "ho256": dict(kind="ho", n_max=255, omega=pi, gamma=pi, dt=1 / 1440, f_max=5.0, ci=80, seed=1256,
                  kp=0.0, kd=1.5),
    "qo171": dict(kind="grid", x_max=8.5, h=0.1, lam=0.04 * pi, mass=1 / pi, gamma=0.01 * pi, dt=1 / 1440,
                  f_max=5.0, ci=80, seed=2171, kp=0.0, kd=1.0, k0=0.2),
    "iqo513": dict(kind="grid", x_max=12.8, h=0.05, lam=-0.01 * pi, mass=1 / pi, gamma=pi, dt=1 / 2880,
                   f_max=5.0, ci=160, seed=3513, kp=1.0, kd=1.0, k0=0.0),
}


# planted zero words (u1 = 0 / u2 = 0 of a Box-Muller pair): (seed, words drawn before, zeroed offsets)
ZERO_CASES = [(5, 6, (0,)), (6, 6, (3,)), (7, 622, (0,)), (8, 620, (0, 2)), (9, 2, (0, 1))]


def stream_child(out_path: str):
    d = {name: M.vsl_gaussian(c["seed"], 2 * STEPS) for name, c in CASES.items()}
    for i, (seed, k, zs) in enumerate(ZERO_CASES):
        d[f"zero{i}_state"], d[f"zero{i}_normals"] = M.vsl_planted_zero(seed, k, zs, 8)
    np.savez(out_path, **d)


def cnr_streams():
    path = "/tmp/_mkl_v2_cnr.npz"
    subprocess.check_call([sys.executable, __file__, "--stream-child", path],
                          env={**os.environ, "MKL_CBWR": "COMPATIBLE"})
    with np.load(path) as z:
        res = {k: z[k] for k in z.files}
    os.unlink(path)
    return res


def psi0_of(name, c, sim):
    if c["kind"] == "ho":      # a coherent state |alpha = 2>
        a = 2.0
        amp = np.zeros(c["n_max"] + 1, np.complex128)
        amp[0] = np.exp(-a * a / 2)
        for k in range(1, len(amp)):
            amp[k] = amp[k - 1] * a / sqrt(k)
        return amp
    # the drivers' Gaussian_packet(wavelength = 1 / k0, mean 0, std 1) (QO/main_parallel.py:177-181,
    # IQO/main_parallel.py:182-183) on the module's grid
    x = sim.x
    return (np.exp(2.j * pi * x * c["k0"]) * np.exp(-x * x / 4.) / sqrt(sqrt(2 * pi))).astype(np.complex128)


def action_of(c, xs):
    """PD rule on <x> at the control step (F = -(kp x + kd dx/dt)), on the 21 force levels."""
    ci, dt = c["ci"], c["dt"]
    x1 = xs[-1]
    x0 = xs[-1 - ci] if len(xs) > ci else x1
    v = (x1 - x0) / (ci * dt)
    a = int(np.clip(np.round(-(c["kp"] * x1 + c["kd"] * v) / (c["f_max"] / 10.)), -10, 10))
    return 10 + a


def run_case(name, c, r):
    if c["kind"] == "ho":
        sim = M.HoMkl(c["n_max"], c["omega"])
    else:
        sim = M.GridMkl(c["x_max"], c["h"], c["lam"], c["mass"])
    psi = psi0_of(name, c, sim)
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
    print(f"{name}: N={sim.N} |<x>| max {np.abs(xs).max():.3f}, actions {sorted(set(acts.tolist()))}, "
          f"fails {sum(fs)}")
    return out


def main():
    if not M.available():
        sys.exit(f"MKL runtime not found at {M.MKL_PATH}")
    streams = cnr_streams()
    data = {}
    for name, c in CASES.items():
        data.update(run_case(name, c, streams[name].reshape(STEPS, 2)))
    data["zero/cases"] = np.array(json.dumps(ZERO_CASES).encode())
    data["zero/state"] = np.stack([streams[f"zero{i}_state"] for i in range(len(ZERO_CASES))])
    data["zero/normals"] = np.stack([streams[f"zero{i}_normals"] for i in range(len(ZERO_CASES))])
    print("zero-word normals:", data["zero/normals"][:, :2])
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
