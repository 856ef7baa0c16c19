"""The oracle pinned at the reference's MKL boundary, CPU.

Fixtures: tests/golden/mkl_v1.npz, made by tests/golden/make_mkl_fixtures.py from the MKL 2021.4
runtime the reference links, through the reference's own call sequences (tests/golden/mklref.py).
"""
from __future__ import annotations

import json
import os
from math import pi

import numpy as np
import pytest

from oracle import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = os.path.join(HERE, "golden", "mkl_v1.npz")


@pytest.fixture(scope="module")
def fx():
    with np.load(FIX) as z:
        return {k: z[k] for k in z.files}


# ---- H3: the noise stream (set_seed IHO/simulation_i.cpp:574-579, vdRngGaussian :435)
def test_mt19937_words_equal_mkl(fx):
    """vslNewStream(VSL_BRNG_MT19937, seed) = mt19937ar init_by_array({seed}): every word, every seed
    (0, 2^31 + 5 and 2^32 - 1 included), over several twists."""
    for s, words in zip(fx["stream/seeds"], fx["stream/words"]):
        assert np.array_equal(O.MT19937(int(s)).words(len(words)), words), int(s)
    lw = fx["stream/long_words"]
    assert np.array_equal(O.MT19937(int(fx["stream/long_seed"])).words(len(lw)), lw)


def test_boxmuller_equals_mkl_compatible_path(fx):
    """VSL_RNG_METHOD_GAUSSIAN_BOXMULLER: x = sqrt(-2 ln u1) sin(2 pi u2), u = word * 2^-32, two words
    per normal, drawn 2 per step: equal to MKL's MKL_CBWR=COMPATIBLE output to <= 2 ulp (libm vs MKL's
    accurate-path rounding; 1 value in 7 000 differs by 2 ulp)."""
    for s, ref in zip(fx["stream/seeds"], fx["stream/cnr/normals"]):
        got = O.MT19937(int(s)).normals(len(ref))
        assert np.all(np.abs(got - ref) <= 2 * np.spacing(np.abs(ref))), int(s)
    ref = fx["stream/cnr/long"]
    got = O.MT19937(int(fx["stream/long_seed"])).normals(len(ref))
    assert np.all(np.abs(got - ref) <= 2 * np.spacing(np.abs(ref)))


def test_mkl_default_path_is_reduced_accuracy(fx):
    """MKL's default dispatch evaluates the transform in its enhanced-performance vector math: within
    5e-8 of the exact formula, and not even the same numbers on AVX2 and AVX-512 — the reference's own
    noise is a property of the host CPU at that level."""
    d, a2, c = fx["stream/default/normals"], fx["stream/avx2/normals"], fx["stream/cnr/normals"]
    assert 0 < np.abs(d - c).max() < 5e-8
    assert 0 < np.abs(a2 - c).max() < 5e-8
    assert np.abs(d - a2).max() > 0


# ---- H4: band LU (reset_ab IHO:249-251, QO:410-411) and the solve (IHO:487, QO:622)
def _lu_case(fx, name):
    c = json.loads(bytes(fx[f"lu/{name}/params"]).decode())
    if c["kind"] == "fock":
        s = O.OracleSystem(O.IHO, n_max=c["n_max"], omega=c["omega"])
    else:
        fam = O.IQO if c["lam"] < 0 else O.QO
        s = O.OracleSystem(fam, x_max=c["x_max"], grid_size=c["h"], lambda_=c["lam"], mass=c["mass"])
    return c, s


@pytest.mark.parametrize("name", ["iho512", "iqo513", "qo1025"])
def test_band_lu_pivots_factors_and_solves_equal_mkl(fx, name):
    c, s = _lu_case(fx, name)
    ipiv = fx[f"lu/{name}/ipiv"]
    n = ipiv.shape[1]
    assert s.N == n
    # no row interchange at any of the 21 forces: the pivot-free device LU is exact (H4)
    assert np.array_equal(ipiv, np.tile(np.arange(1, n + 1, dtype=np.int32), (21, 1)))
    for k, a in enumerate(fx[f"lu/{name}/lu_slots"]):
        F = (int(a) - 10) * (c["f_max"] / 10.)
        ab, ip, _ = s.tab_export(c["dt"], F)
        assert np.array_equal(ip + 1, ipiv[a])
        mkl_lu = fx[f"lu/{name}/lu"][k]
        err = np.abs(ab.T - mkl_lu).max() / np.abs(mkl_lu).max()
        assert err < 1e-15, (a, err)
    rhs = fx[f"lu/{name}/rhs"]
    for k, a in enumerate(fx[f"lu/{name}/sol_slots"]):
        F = (int(a) - 10) * (c["f_max"] / 10.)
        x = s.tab_solve(c["dt"], F, rhs)
        ref = fx[f"lu/{name}/sol"][k]
        assert np.abs(x - ref).max() / np.abs(ref).max() < 1e-14, a


# ---- H1: term7 = A . D1 under MKL's {HERMITIAN, UPPER} descriptor (IHO:23, :551)
@pytest.mark.parametrize("a", [0, 3, 10, 20])
def test_term7_hermitian_descriptor_equals_mkl(fx, a):
    """A as MKL builds it (spmm / z_add chain with the SYMMETRIC hint, IHO:253-272) equals the oracle's
    band; the oracle's reference-mode term7 (upper triangle + conjugate mirror, stored complex
    diagonal kept) equals mkl_sparse_z_mv with the reference's descriptor; the intended
    complex-symmetric A (a_mode 1) does not."""
    n_max = int(fx["mv/n_max"])
    dt, F = 1.0 / 1440, (a - 10) * 0.8
    ref_mode = O.OracleSystem(O.IHO, n_max=n_max, omega=pi, a_mode=0)
    exact = O.OracleSystem(O.IHO, n_max=n_max, omega=pi, a_mode=1)
    _, _, A = ref_mode.tab_export(dt, F)
    Am = fx[f"mv/a{a}/A_band"]
    assert np.abs(A - Am).max() / np.abs(Am).max() < 1e-15
    for k, v in enumerate(fx["mv/v"]):
        y = fx[f"mv/a{a}/y"][k]
        got = ref_mode.term7(dt, F, v)
        assert np.abs(got - y).max() <= 1e-14 * np.abs(y).max(), k
        other = exact.term7(dt, F, v)
        assert np.abs(other - y).max() > 1e-6 * np.abs(y).max()


# ---- H2: the quartic p_hat - pbar I with the DIAG_UNIT identity copy (QO:170-178, :337)
@pytest.mark.parametrize("name", ["iqo521", "qo1025"])
def test_grid_p_relative_equals_mkl(fx, name):
    x_max, h, pbar = fx[f"pgrid/{name}/params"]
    fam = O.IQO if name.startswith("iqo") else O.QO
    s = O.OracleSystem(fam, x_max=x_max, grid_size=h, lambda_=0.04 * pi, mass=1 / pi)
    v, y = fx[f"pgrid/{name}/v"], fx[f"pgrid/{name}/y"]
    got = s.grid_p_apply(v, pbar)
    assert np.abs(got - y).max() <= 1e-13 * np.abs(y).max()


# ---- the whole go_one_step in MKL call order vs the oracle, 1000 steps on the reference's stream
@pytest.mark.parametrize("name", ["iho181", "iho512"])
def test_oracle_tracks_mkl_ordered_stepper(fx, name):
    """mklref.IhoMkl (every cblas / sparse / LAPACKE call of go_one_step in the reference's order) and
    the oracle, fed the same MKL noise (CBWR=COMPATIBLE stream of the case's seed) and actions, agree
    to 1e-9 in psi after 1000 steps and in every step's (q, x_mean, Fail); the oracle's own
    MT19937 stream reproduces the same trajectory."""
    n_max = int(fx[f"traj/{name}/n_max"])
    dt, gamma, f_max = fx[f"traj/{name}/phys"]
    acts = fx[f"traj/{name}/actions"]
    s = O.OracleSystem(O.IHO, n_max=n_max, omega=pi)
    for source in ("fixture", "oracle_mt"):
        if source == "fixture":
            r = fx[f"traj/{name}/cnr/noise"]
        else:
            r = O.MT19937(int(fx[f"traj/{name}/seed"])).normals(2 * len(fx[f"traj/{name}/cnr/q"])).reshape(-1, 2)
        psi = np.zeros((1, n_max + 1), np.complex128)
        psi[0, 0] = 1.0
        qs, xs = [], []
        k0 = 0
        for c, a in enumerate(acts):
            n = min(80, len(r) - k0)
            fail, q, xm = s.run_batch(psi, np.array([a], np.int32), f_max, n, dt, gamma,
                                      noise=r[k0:k0 + n].reshape(n, 1, 2), want_q=True, n_threads=1)
            assert fail[0] == 0
            qs.append(q[:, 0])
            xs.append(xm[:, 0])
            k0 += n
        q, xm = np.concatenate(qs), np.concatenate(xs)
        assert np.abs(q - fx[f"traj/{name}/cnr/q"]).max() < 1e-9
        assert np.abs(xm - fx[f"traj/{name}/cnr/x_mean"]).max() < 1e-9
        final = fx[f"traj/{name}/cnr/psi"][-1]
        err = np.linalg.norm(psi[0] - final)
        assert err < 1e-9, (source, err)
    assert not fx[f"traj/{name}/cnr/fail"].any()


def test_default_mkl_stream_trajectory_deviation_is_bounded(fx):
    """The same trajectory on MKL's default (AVX-512, reduced-accuracy) normals: the <= 5e-8 noise
    difference stays a small, bounded trajectory difference (documented, not a parity claim)."""
    for name in ("iho181", "iho512"):
        a = fx[f"traj/{name}/cnr/psi"][-1]
        b = fx[f"traj/{name}/default/psi"][-1]
        d = np.linalg.norm(a - b)
        assert 0 < d < 1e-5, (name, d)


# ---- mkl_v2.npz: the harmonic and grid modules' go_one_step and compute_statistics in MKL call order
FIX2 = os.path.join(HERE, "golden", "mkl_v2.npz")
V2_CASES = ["ho71", "ho256", "qo171", "iqo513"]


@pytest.fixture(scope="module")
def fx2():
    with np.load(FIX2) as z:
        return {k: z[k] for k in z.files}


def v2_system(fx2, name):
    c = json.loads(bytes(fx2[f"traj/{name}/params"]).decode())
    if c["kind"] == "ho":
        return c, O.OracleSystem(O.HO, n_max=c["n_max"], omega=c["omega"])
    fam = O.IQO if c["lam"] < 0 else O.QO
    return c, O.OracleSystem(fam, x_max=c["x_max"], grid_size=c["h"], lambda_=c["lam"], mass=c["mass"])


@pytest.mark.parametrize("name", V2_CASES)
def test_oracle_tracks_mkl_ordered_stepper_v2(fx2, name):
    """mklref.HoMkl / GridMkl (HO/simulation.cpp:413-470,527-554; QO/simulation_quart.cpp:394-432,
    :434-486, :569-644 with its SYMMETRIC / DIAGONAL descriptors) and the oracle, fed the same MKL noise
    and actions from the same psi0, agree to 1e-9 in psi (grid: weighted by sqrt(h)) at steps 100 / 500 /
    1000 and in every step's q and x_mean; Fail is never raised; the oracle's own MT19937 stream of the
    case's seed reproduces the trajectory; and on the grid the oracle's 20 moments of each MKL snapshot
    equal compute_statistics' (QO:326-362) to 1e-9 relative. (psi is compared at step 1000; the 100 /
    500 snapshots fall inside control intervals and are checked by the GPU drop-in test.)"""
    c, s = v2_system(fx2, name)
    acts, ci = fx2[f"traj/{name}/actions"], c["ci"]
    w = np.sqrt(c["h"]) if c["kind"] == "grid" else 1.0
    for source in ("fixture", "oracle_mt"):
        if source == "fixture":
            r = fx2[f"traj/{name}/noise"]
        else:
            r = O.MT19937(int(c["seed"])).normals(2 * len(fx2[f"traj/{name}/q"])).reshape(-1, 2)
        psi = fx2[f"traj/{name}/psi0"].copy().reshape(1, -1)
        qs, xs, snaps = [], [], []
        k0 = 0
        for a in acts:
            n = min(ci, len(r) - k0)
            fail, q, xm = s.run_batch(psi, np.array([a], np.int32), c["f_max"], n, c["dt"], c["gamma"],
                                      noise=r[k0:k0 + n].reshape(n, 1, 2), want_q=True, n_threads=1)
            assert fail[0] == 0
            qs.append(q[:, 0])
            xs.append(xm[:, 0])
            k0 += n
        q, xm = np.concatenate(qs), np.concatenate(xs)
        assert np.abs(q - fx2[f"traj/{name}/q"]).max() < 1e-9, source
        assert np.abs(xm - fx2[f"traj/{name}/x_mean"]).max() < 1e-9, source
        err = np.linalg.norm(psi[0] - fx2[f"traj/{name}/psi"][-1]) * w
        assert err < 1e-9, (source, err)
    assert not fx2[f"traj/{name}/fail"].any()
    if c["kind"] == "grid":
        for snap, ref in zip(fx2[f"traj/{name}/psi"], fx2[f"traj/{name}/moments"]):
            got = s.moments(snap)
            assert got.shape == (20,)
            assert np.abs(got - ref).max() <= 1e-9 * max(1.0, np.abs(ref).max())


def test_boxmuller_zero_word_equals_mkl(fx2):
    """A zero first word (u1 = 0, 2^-32 per normal): MKL's BOXMULLER gives the finite radius
    3.4244955099270222, not an infinite normal. States with planted zero words (saved / loaded through
    vslSaveStreamM / vslLoadStreamM, make_mkl_fixtures_v2.py): the oracle's next 8 normals equal MKL's
    CBWR=COMPATIBLE output to <= 2 ulp, the zero-word ones included (and zero second words give 0)."""
    for st, ref in zip(fx2["zero/state"], fx2["zero/normals"]):
        mt = O.MT19937(0)
        mt.st[:] = st
        got = mt.normals(len(ref))
        assert np.all(np.isfinite(got))
        assert np.all(np.abs(got - ref) <= 2 * np.spacing(np.abs(ref))), (got, ref)


# ---- mkl_v3.npz: the same MKL-call-ordered pin at the large configurations' sizes (C3's x_n = 1025 grid at
# dt 1/11520, IHO N = 1024 and C5's N = 2048; make_mkl_fixtures_v3.py)
FIX3 = os.path.join(HERE, "golden", "mkl_v3.npz")
V3_CASES = ["qo1025", "iho1024", "iho2048"]


@pytest.fixture(scope="module")
def fx3():
    with np.load(FIX3) as z:
        return {k: z[k] for k in z.files}


@pytest.mark.parametrize("name", V3_CASES)
def test_oracle_tracks_mkl_ordered_stepper_v3(fx3, name):
    """mklref.GridMkl at QO x_n = 1025 (QO/simulation_quart.cpp:394-432,569-644) and mklref.IhoMkl at
    IHO N = 1024 / 2048 (IHO/simulation_i.cpp:227-277,432-489), fed MKL's CBWR=COMPATIBLE stream of the
    case's seed: the oracle agrees to 1e-9 in psi (grid weighted by sqrt(h)) after 1000 steps and in every
    step's q and x_mean, on the fixture's normals and on its own MT19937 stream; Fail is never raised; the
    grid's 20 moments of each MKL snapshot equal compute_statistics' to 1e-9 relative."""
    c = json.loads(bytes(fx3[f"traj/{name}/params"]).decode())
    if c["kind"] == "iho":
        s = O.OracleSystem(O.IHO, n_max=c["n_max"], omega=c["omega"])
        w = 1.0
    else:
        s = O.OracleSystem(O.QO, x_max=c["x_max"], grid_size=c["h"], lambda_=c["lam"], mass=c["mass"])
        w = np.sqrt(c["h"])
    acts, ci = fx3[f"traj/{name}/actions"], c["ci"]
    assert len(set(acts.tolist())) > 2          # the force changes: several reset_ab tables are exercised
    for source in ("fixture", "oracle_mt"):
        if source == "fixture":
            r = fx3[f"traj/{name}/noise"]
        else:
            r = O.MT19937(int(c["seed"])).normals(2 * len(fx3[f"traj/{name}/q"])).reshape(-1, 2)
        psi = fx3[f"traj/{name}/psi0"].copy().reshape(1, -1)
        qs, xs = [], []
        k0 = 0
        for a in acts:
            n = min(ci, len(r) - k0)
            fail, q, xm = s.run_batch(psi, np.array([a], np.int32), c["f_max"], n, c["dt"], c["gamma"],
                                      noise=r[k0:k0 + n].reshape(n, 1, 2), want_q=True, n_threads=1)
            assert fail[0] == 0
            qs.append(q[:, 0])
            xs.append(xm[:, 0])
            k0 += n
        q, xm = np.concatenate(qs), np.concatenate(xs)
        assert np.abs(q - fx3[f"traj/{name}/q"]).max() < 1e-9, source
        assert np.abs(xm - fx3[f"traj/{name}/x_mean"]).max() < 1e-9, source
        err = np.linalg.norm(psi[0] - fx3[f"traj/{name}/psi"][-1]) * w
        assert err < 1e-9, (source, err)
    assert not fx3[f"traj/{name}/fail"].any()
    if c["kind"] == "grid":
        for snap, ref in zip(fx3[f"traj/{name}/psi"], fx3[f"traj/{name}/moments"]):
            got = s.moments(snap)
            assert np.abs(got - ref).max() <= 1e-9 * max(1.0, np.abs(ref).max())
