"""Generate tests/golden/mkl_v1.npz: fixtures from the MKL runtime the reference links (mklref.py).

    python tests/golden/make_mkl_fixtures.py          (needs /opt/conda/lib/libmkl_rt.so; this container)

Contents (every array is data: inputs and MKL's outputs; no reference source is involved):
  stream/*   vslNewStream(VSL_BRNG_MT19937, seed) uniform words (viRngUniformBits) and the reference's
             vdRngGaussian(BOXMULLER, stream, 2, r) normals under three MKL code paths: the default
             dispatch of this CPU (AVX-512), MKL_ENABLE_INSTRUCTIONS=AVX2, MKL_CBWR=COMPATIBLE
  lu/<case>  LAPACKE_zgbtrf pivots for all 21 forces, the LU band of three of them, and zgbtrs
             solutions of a fixed right-hand side (IHO N=512, IQO x_n=513, QO x_n=1025)
  mv/*       the IHO correction factor A built by the reference's spmm / z_add chain (IHO:253-272) as
             MKL holds it, and term7 = mkl_sparse_z_mv(A, {HERMITIAN, UPPER}) of fixed vectors (:551)
  pgrid/*    the quartic (p̂ - p̄ I) v with the {HERMITIAN, UPPER, DIAG_UNIT} identity (QO:170-178,337)
  traj/<case>  IHO trajectories of the MKL-call-ordered stepper (mklref.IhoMkl): psi0 = |0>, 1000 steps,
             actions per 80-step interval, noise = the reference's stream for `seed` under both the
             CBWR=COMPATIBLE and the default MKL paths; psi after 100/500/1000 steps, q, x_mean, Fail
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
from math import pi

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)

import mklref as M  # noqa: E402

OUT = os.path.join(HERE, "mkl_v1.npz")
SEEDS = [0, 1, 7, 42, 99998, 2147483653, 4294967295]
N_WORDS, N_NORMALS = 1400, 1000
LONG_SEED, LONG_NORMALS = 12345, 4000          # several twists of one stream
STEPS, CI = 1000, 80
# iho181: the IHO driver's own n_max (IHO/arguments.py); iho512: the metric's N. At N = 512 the reference
# scheme with dt = 1/1440 amplifies rounding in the top Fock levels until it blows up after ~700 steps
# (MKL stepper and oracle alike), so that case runs at dt = 1/2880 (README rule: smaller dt for larger N)
TRAJ = {"iho512": dict(n_max=511, seed=4242, dt=1.0 / 2880), "iho181": dict(n_max=180, seed=77, dt=1.0 / 1440)}
IHO_DT, IHO_GAMMA, IHO_FMAX = 1.0 / 1440, 2 * pi, 8.0   # IHO/arguments.py:6-17 (gamma * pi)


def stream_child(out_path: str):
    data = {}
    for s in SEEDS:
        data[f"g{s}"] = M.vsl_gaussian(s, N_NORMALS)
    data["long"] = M.vsl_gaussian(LONG_SEED, LONG_NORMALS)
    for name, t in TRAJ.items():
        data[f"traj_{name}"] = M.vsl_gaussian(t["seed"], 2 * STEPS)
    np.savez(out_path, **data)


def stream_modes():
    modes = {"default": {}, "avx2": {"MKL_ENABLE_INSTRUCTIONS": "AVX2"}, "cnr": {"MKL_CBWR": "COMPATIBLE"}}
    res = {}
    for mode, env in modes.items():
        path = f"/tmp/_mkl_stream_{mode}.npz"
        subprocess.check_call([sys.executable, __file__, "--stream-child", path], env={**os.environ, **env})
        with np.load(path) as z:
            res[mode] = {k: z[k] for k in z.files}
        os.unlink(path)
    return res


def lu_cases():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import refmath as RM
    cases = {
        "iho512": dict(kind="fock", n_max=511, omega=pi, f_max=8.0, dt=1.0 / 1440, kl=2),
        "iqo513": dict(kind="grid", x_max=12.8, h=0.05, lam=-0.01 * pi, mass=1 / pi, f_max=5.0, dt=1.0 / 2880, kl=4),
        "qo1025": dict(kind="grid", x_max=8.5, h=8.5 / 512, lam=0.04 * pi, mass=1 / pi, f_max=5.0, dt=1.0 / 1440, kl=4),
    }
    out = {}
    rng = np.random.default_rng(2024)
    for name, c in cases.items():
        if c["kind"] == "fock":
            ops = RM.fock_ops(c["n_max"], c["omega"], inverted=True)
            H, X, cc = ops["H"], ops["x"], c["omega"]
        else:
            g = RM.grid_ops(c["x_max"], c["h"], c["lam"], c["mass"])
            H, X, cc = g["H"], g["X"], pi
        n, kl = H.shape[0], c["kl"]
        rhs = rng.standard_normal(n) + 1j * rng.standard_normal(n)
        ipivs, lus, sols = [], {}, {}
        for a in range(21):
            F = (a - 10) * (c["f_max"] / 10.)
            ab = M.band_rows(np.eye(n) + 0.5j * c["dt"] * (H - cc * F * X), kl)
            lu, ipiv = M.band_lu(ab, kl)
            ipivs.append(ipiv)
            if a in (0, 20):
                lus[a] = lu
            if a in (0, 7, 13, 20):
                sols[a] = M.band_solve(lu, ipiv, kl, rhs)
        out[f"lu/{name}/params"] = np.array(json.dumps({k: v for k, v in c.items()}).encode())
        out[f"lu/{name}/ipiv"] = np.stack(ipivs)
        out[f"lu/{name}/lu_slots"] = np.array(sorted(lus))
        out[f"lu/{name}/lu"] = np.stack([lus[a] for a in sorted(lus)])
        out[f"lu/{name}/rhs"] = rhs
        out[f"lu/{name}/sol_slots"] = np.array(sorted(sols))
        out[f"lu/{name}/sol"] = np.stack([sols[a] for a in sorted(sols)])
    return out


def mv_cases():
    out = {}
    rng = np.random.default_rng(7)
    n_max = 511
    sim = M.IhoMkl(n_max, pi)
    v = rng.standard_normal((2, n_max + 1)) + 1j * rng.standard_normal((2, n_max + 1))
    v[1, 40:] = 0.0                         # a low-level state, like the controlled cartpole's D1
    for a in (0, 3, 10, 20):
        F = (a - 10) * (IHO_FMAX / 10.)
        sim.reset_ab(IHO_DT, F)
        Ad = sim.A.dense()
        bw = 10
        band = np.zeros((2 * bw + 1, n_max + 1), np.complex128)   # band[d + bw][i] = A[i][i + d]
        for d in range(-bw, bw + 1):
            for i in range(max(0, -d), min(n_max + 1, n_max + 1 - d)):
                band[d + bw][i] = Ad[i, i + d]
        assert np.count_nonzero(Ad) == np.count_nonzero(band), "A wider than 21 bands"
        ys = []
        for k in range(2):
            y = np.zeros(n_max + 1, np.complex128)
            sim.A.mv(complex(1., 0.), sim.descr, np.ascontiguousarray(v[k]), complex(0., 0.), y)
            ys.append(y)
        out[f"mv/a{a}/A_band"] = band
        out[f"mv/a{a}/y"] = np.stack(ys)
    out["mv/v"] = v
    out["mv/n_max"] = np.array(n_max)
    # pgrid: IQO driver grid (x_max 13, h 0.05 -> x_n 521) and C3's QO x_n 1025
    for name, (x_max, h) in {"iqo521": (13.0, 0.05), "qo1025": (8.5, 8.5 / 512)}.items():
        x_n = 2 * int(x_max / h + 0.5) + 1
        w = rng.standard_normal(x_n) + 1j * rng.standard_normal(x_n)
        pbar = 0.37
        out[f"pgrid/{name}/params"] = np.array([x_max, h, pbar])
        out[f"pgrid/{name}/v"] = w
        out[f"pgrid/{name}/y"] = M.grid_p_relative(x_n, h, pbar, w)
    return out


def feedback_action(xm_hist, dt: float) -> int:
    """A PD rule on <x> at the control step, |F| <= 4 (keeps the cartpole up for the 1000 steps, so the
    whole trajectory stays physical): F = -(1.3 x + 0.1 dx/dt)."""
    x1 = xm_hist[-1]
    x0 = xm_hist[-1 - CI] if len(xm_hist) > CI else x1
    v = (x1 - x0) / (CI * dt)
    a = 10 - int(np.clip(np.round((1.3 * x1 + 0.1 * v) / (IHO_FMAX / 10.)), -5, 5))
    return int(a)


def traj_cases(streams):
    out = {}
    for name, t in TRAJ.items():
        acts = np.full((STEPS + CI - 1) // CI, 10, np.int32)   # no control in the first interval
        out[f"traj/{name}/n_max"] = np.array(t["n_max"])
        out[f"traj/{name}/seed"] = np.array(t["seed"])
        dt = t["dt"]
        out[f"traj/{name}/phys"] = np.array([dt, IHO_GAMMA, IHO_FMAX])
        for mode in ("cnr", "default"):   # the cnr run decides the actions; the default run replays them
            r = streams[mode][f"traj_{name}"].reshape(STEPS, 2)
            sim = M.IhoMkl(t["n_max"], pi)
            psi = np.zeros(t["n_max"] + 1, np.complex128)
            psi[0] = 1.0
            qs, xs, fs, snaps = [], [], [], []
            for k in range(STEPS):
                F = (int(acts[k // CI]) - 10) * (IHO_FMAX / 10.)
                q, xm, f = sim.step(psi, dt, F, IHO_GAMMA, r[k])
                qs.append(q)
                xs.append(xm)
                fs.append(f)
                if k + 1 in (100, 500, 1000):
                    snaps.append(psi.copy())
                if mode == "cnr" and (k + 1) % CI == 0 and (k + 1) // CI < len(acts):
                    acts[(k + 1) // CI] = feedback_action(xs, dt)
            out[f"traj/{name}/{mode}/psi"] = np.stack(snaps)
            out[f"traj/{name}/{mode}/q"] = np.array(qs)
            out[f"traj/{name}/{mode}/x_mean"] = np.array(xs)
            out[f"traj/{name}/{mode}/fail"] = np.array(fs, np.int8)
            out[f"traj/{name}/{mode}/noise"] = r
            out[f"traj/{name}/actions"] = acts.copy()
            print(f"traj {name} {mode}: |<x>| max {np.abs(xs).max():.3f}, fails {sum(fs)}")
    return out


def main():
    if not M.available():
        sys.exit(f"MKL runtime not found at {M.MKL_PATH}")
    streams = stream_modes()
    data = {}
    data["stream/seeds"] = np.array(SEEDS, np.uint64)
    data["stream/words"] = np.stack([M.vsl_bits(s, N_WORDS) for s in SEEDS])
    data["stream/long_seed"] = np.array(LONG_SEED)
    data["stream/long_words"] = M.vsl_bits(LONG_SEED, 2 * LONG_NORMALS)
    for mode, d in streams.items():
        data[f"stream/{mode}/normals"] = np.stack([d[f"g{s}"] for s in SEEDS])
        data[f"stream/{mode}/long"] = d["long"]
    data.update(lu_cases())
    data.update(mv_cases())
    data.update(traj_cases(streams))
    data["meta"] = np.array(json.dumps({
        "mkl": "2021.4.0 (/opt/conda/lib/libmkl_rt.so, conda mkl-2021.4.0-h06a4308_640)",
        "default_path_cpu": open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].strip(": \t"),
    }).encode())
    np.savez_compressed(OUT, **data)
    print(f"wrote {OUT}: {len(data)} arrays, {os.path.getsize(OUT)} bytes")


if __name__ == "__main__":
    if len(sys.argv) == 3 and sys.argv[1] == "--stream-child":
        stream_child(sys.argv[2])
    else:
        main()
