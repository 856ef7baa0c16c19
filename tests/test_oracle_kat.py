"""Pin the CPU restatement (oracle/) with known-answer tests.

The reference binary never ran (denied; the reference has no tests or fixtures, §4); its
MKL boundary is pinned in tests/test_mkl_fixtures.py. These tests pin the restatement against independent physics and
against dense numpy restatements of the reference's own Python operator definitions.
"""
from math import pi, sqrt

import numpy as np
import pytest
import scipy.linalg as sl

from tests import refmath as R

DT = 1 / 1440


# ---- Philox4x32-10 known-answer vectors (Random123 kat_vectors) -------------------------------
@pytest.mark.parametrize("ctr,key,out", [
    ([0, 0, 0, 0], [0, 0], [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]),
    ([0xffffffff] * 4, [0xffffffff] * 2, [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]),
    ([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0],
     [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]),
])
def test_philox_kat(oracle_mod, ctr, key, out):
    assert list(oracle_mod.philox(ctr, key)) == out


def test_normals_distribution(oracle_mod):
    r = np.array([oracle_mod.normals(42, e, k) for e in range(40) for k in range(100)])
    assert abs(r.mean()) < 0.05 and abs(r.std() - 1) < 0.05
    assert abs(np.corrcoef(r[:, 0], r[:, 1])[0, 1]) < 0.06


# ---- operators against the reference's Python definitions ------------------------------------
@pytest.mark.parametrize("fam", [0, 1])
def test_fock_operators(oracle_mod, fam):
    s = oracle_mod.OracleSystem(fam, n_max=40, omega=pi)
    ops = R.fock_ops(40, pi, inverted=(fam == 1))
    np.testing.assert_allclose(s.dense_x(), ops["x"], rtol=0, atol=1e-14)
    np.testing.assert_allclose(s.dense_h(), ops["H"], rtol=1e-15, atol=1e-12)


@pytest.mark.parametrize("fam,lam", [(2, 0.04 * pi), (3, -0.01 * pi)])
def test_grid_operators(oracle_mod, fam, lam):
    s = oracle_mod.OracleSystem(fam, x_max=3.0, grid_size=0.1, lambda_=lam, mass=1 / pi)
    g = R.grid_ops(3.0, 0.1, lam, 1 / pi)
    assert s.N == g["n"] == 61
    np.testing.assert_allclose(np.diag(s.dense_x()), g["x"], atol=1e-14)
    np.testing.assert_allclose(s.dense_h(), g["H"], rtol=1e-13, atol=1e-9)


# ---- band LU: no pivoting at the reference parameters, LU reproduces ab ----------------------
@pytest.mark.parametrize("fam,kw,dt,fmax", [
    (0, dict(n_max=70), DT, 5.0),
    (1, dict(n_max=180), DT, 8.0),
    (1, dict(n_max=511), DT, 8.0),
    (2, dict(x_max=8.5, grid_size=0.1, lambda_=0.04 * pi, mass=1 / pi), DT, 5.0),
    (3, dict(x_max=12.8, grid_size=0.05, lambda_=-0.01 * pi, mass=1 / pi), 1 / 2880, 5.0),
])
def test_no_pivoting_at_reference_parameters(oracle_mod, fam, kw, dt, fmax):
    s = oracle_mod.OracleSystem(fam, **kw)
    for a in (0, 3, 10, 17, 20):
        assert s.n_swaps(dt, (a - 10) * (fmax / 10)) == 0


def test_band_lu_reconstructs_matrix(oracle_mod):
    s = oracle_mod.OracleSystem(1, n_max=30)
    F = 2.4
    ab, ipiv, _ = s.tab_export(DT, F)
    N, kl = s.N, 2
    ldab = ab.shape[1]
    L = np.eye(N, dtype=complex)
    U = np.zeros((N, N), dtype=complex)
    for j in range(N):
        for i in range(max(0, j - 2 * kl), min(N, j + kl + 1)):
            row = 2 * kl + i - j
            if i <= j:
                U[i, j] = ab[j, row]
            else:
                L[i, j] = ab[j, row]
    assert np.all(ipiv == np.arange(N))
    HF = s.dense_h() - pi * F * s.dense_x()
    M = np.eye(N) + 1j * DT / 2 * HF
    np.testing.assert_allclose(L @ U, M, atol=1e-15)
    assert ldab == 3 * kl + 1


# ---- unitary limit (gamma = 0): the scheme is exp(-i H_F dt) to O(dt^7) -----------------------
@pytest.mark.parametrize("fam,kw,F", [
    (0, dict(n_max=40), 2.0),
    (1, dict(n_max=40), 3.2),
    (2, dict(x_max=6.0, grid_size=0.1, lambda_=0.04 * pi, mass=1 / pi), 1.5),
    (3, dict(x_max=6.0, grid_size=0.1, lambda_=-0.01 * pi, mass=1 / pi), -2.5),
])
def test_unitary_limit_matches_expm(oracle_mod, fam, kw, F):
    s = oracle_mod.OracleSystem(fam, a_mode=1, **kw)
    if fam < 2:
        psi = s.fock_random_state(1234, 3, 12)
        c = pi
    else:
        psi = s.gaussian_packet(0.2, 0.3, 0.7)   # smooth inside the box: no edge-truncation high-k content
        psi /= np.linalg.norm(psi) * sqrt(s.params.grid_size)   # the reference renormalises each step
        c = pi
    HF = s.dense_h() - c * F * s.dense_x()
    p = psi.copy()
    n = 40
    for _ in range(n):
        s.step(p, DT, F, 0.0, [0.7, -1.1])
    ref = sl.expm(-1j * HF * DT * n) @ psi
    nrm = sqrt(s.params.grid_size) if fam >= 2 else 1.0
    assert np.linalg.norm((p - ref) * nrm) < 5e-9


def test_mirror_semantics_is_what_differs(oracle_mod):
    """IHO a_mode=0 (MKL HERMITIAN descriptor, App. C H1) departs from exp(-iHdt); a_mode=1 does not."""
    out = {}
    for am in (0, 1):
        s = oracle_mod.OracleSystem(1, n_max=40, a_mode=am)
        psi = s.fock_random_state(7, 0, 12)
        HF = s.dense_h() - pi * 3.2 * s.dense_x()
        p = psi.copy()
        for _ in range(20):
            s.step(p, DT, 3.2, 0.0, [0.0, 0.0])
        out[am] = np.linalg.norm(p - sl.expm(-1j * HF * DT * 20) @ psi)
    assert out[1] < 1e-10 < 1e-7 < out[0]


# ---- full stochastic step against the dense restatement of Appendix A --------------------------
@pytest.mark.parametrize("fam,kw,F,gamma,dt,amode", [
    (0, dict(n_max=30), 1.5, pi, DT, 0),
    (1, dict(n_max=30), -2.4, 2 * pi, DT, 0),
    (1, dict(n_max=30), -2.4, 2 * pi, DT, 1),
    (2, dict(x_max=3.0, grid_size=0.1, lambda_=0.04 * pi, mass=1 / pi), 1.0, 0.01 * pi, DT, 0),
    (3, dict(x_max=3.0, grid_size=0.1, lambda_=-0.01 * pi, mass=1 / pi), -1.0, pi, 1 / 2880, 0),
])
def test_step_matches_dense_scheme(oracle_mod, fam, kw, F, gamma, dt, amode):
    s = oracle_mod.OracleSystem(fam, a_mode=amode, **kw)
    fock = fam < 2
    if fock:
        psi = s.fock_random_state(99, 1, 10)
        H, X, c, w = s.dense_h(), s.dense_x(), pi, 1.0
    else:
        psi = s.gaussian_packet(0.1, -0.2, 0.8)
        H, X, c, w = s.dense_h(), s.dense_x(), pi, s.params.grid_size
    HF = H - c * F * X
    A = R.correction_A(HF, dt)
    A_eff = A if amode == 1 else R.mirror(A, hermitian=(fam == 1))
    p = psi.copy()
    ref = psi.copy()
    for k in range(10):
        r = oracle_mod.normals(5, 0, k)
        q, xm, _ = s.step(p, dt, F, gamma, r)
        ref, q2, xm2 = R.dense_step(ref, H, X, F, c, gamma, dt, r, w, A_eff)
        assert abs(xm - xm2) < 1e-12 and abs(q - q2) < 1e-9
    assert np.linalg.norm((p - ref) * sqrt(w)) < 1e-12


def test_norm_and_fail_flag(oracle_mod):
    s = oracle_mod.OracleSystem(1, n_max=40)
    psi = s.fock_random_state(3, 0, 16)
    for k in range(30):
        _, _, f = s.step(psi, DT, 8.0, 2 * pi, oracle_mod.normals(1, 0, k))
        assert f == 0
        assert abs(np.linalg.norm(psi) - 1) < 1e-13
    top = np.zeros(s.N, dtype=complex)
    top[-1] = 1.0
    assert s.boundary_fail(top) == 1
    g = oracle_mod.OracleSystem(3, x_max=3.0, grid_size=0.1, lambda_=-0.01 * pi, mass=1 / pi)
    edge = np.zeros(g.N, dtype=complex)
    edge[2] = 1.0
    assert g.boundary_fail(edge) == 1


# ---- observations -------------------------------------------------------------------------------
def test_fock_moments_match_python_definition(oracle_mod):
    """get_data_xp (IHO/main_parallel.py:129-131) with the truncated scipy operators."""
    s = oracle_mod.OracleSystem(1, n_max=40)
    ops = R.fock_ops(40, pi)
    psi = s.fock_random_state(11, 2, 14)
    e = lambda op: np.real(np.conj(psi) @ (op @ psi))
    xe, pe = e(ops["x"]), e(ops["p"])
    ref = [xe, pe, e(ops["x2"]) - xe ** 2, e(ops["p2"]) - pe ** 2, e(ops["xppx"]) / 2 - xe * pe]
    np.testing.assert_allclose(s.moments(psi), ref, atol=1e-12)


def test_fock_coherent_state_moments(oracle_mod):
    s = oracle_mod.OracleSystem(0, n_max=60)
    alpha = 1.2 - 0.7j
    n = np.arange(s.N)
    from scipy.special import gammaln
    c = np.exp(-abs(alpha) ** 2 / 2 + n * np.log(alpha + 0j) - 0.5 * gammaln(n + 1))
    m = s.moments(c.astype(np.complex128))
    np.testing.assert_allclose(m, [sqrt(2) * alpha.real, sqrt(2) * alpha.imag, 0.5, 0.5, 0.0], atol=1e-10)


def test_grid_moments_dense_and_gaussian(oracle_mod):
    lam = -0.01 * pi
    s = oracle_mod.OracleSystem(3, x_max=8.0, grid_size=0.05, lambda_=lam, mass=1 / pi)
    g = R.grid_ops(8.0, 0.05, lam, 1 / pi)
    mu, sig, k = 0.4, 0.9, 0.15
    psi = s.gaussian_packet(k, mu, sig)
    m = s.moments(psi)
    np.testing.assert_allclose(m, R.grid_moments_dense(psi, g), rtol=1e-11, atol=1e-11)
    # analytic Gaussian packet: <x>=mu, <p>=2 pi k, Var x = sig^2, Var p = 1/(4 sig^2), odd central 0
    assert abs(m[0] - mu) < 1e-9 and abs(m[1] - 2 * pi * k) < 1e-6
    assert abs(m[2] - sig ** 2) < 1e-9 and abs(m[3]) < 1e-6 and abs(m[4] - 1 / (4 * sig ** 2)) < 1e-5
    assert abs(m[5]) < 1e-9 and abs(m[8]) < 1e-5            # <xxx>, <ppp>
    assert abs(m[9] - 3 * sig ** 4) < 1e-8                   # <xxxx>


def test_outside_probability_window(oracle_mod):
    s = oracle_mod.OracleSystem(3, x_max=12.8, grid_size=0.05, lambda_=-0.01 * pi, mass=1 / pi)
    psi = s.gaussian_packet(0.0, 0.0, 1.0)
    xth = (5.0 / (0.01 * pi) / 4 * pi) ** (1 / 3)
    c, w = s.N // 2, round(xth / 0.05)
    ref = 1.0 - np.sum(np.abs(psi[c - w:c + w]) ** 2) * 0.05
    assert abs(s.outside_prob(psi, xth) - ref) < 1e-15
    assert abs(xth - 5.0) < 1e-12


# ---- the IHO step kernel's X^2 identity (k_step X2H) ----------------------------
@pytest.mark.parametrize("n_max,omega", [(511, pi), (180, pi), (40, 2.0)])
def test_iho_x_squared_is_h_multiple_plus_diagonal(n_max, omega):
    """On the truncated Fock operators of IHO/simulation_i.cpp:65-124, X^2 = -H/omega + diag(d) with
    d_r = X[r][r-1]^2 + X[r][r+1]^2 (the truncation's last row included) — to rounding."""
    ops = R.fock_ops(n_max, omega, inverted=True)
    x, H = ops["x"], ops["H"]
    xu = np.diag(x, 1)
    d = np.concatenate([[0.0], xu ** 2]) + np.concatenate([xu ** 2, [0.0]])
    lhs = x @ x
    rhs = -H / omega + np.diag(d)
    assert np.max(np.abs(lhs - rhs)) <= 1e-15 * np.max(np.abs(lhs))


def test_phi_products_from_s1_s2_s3():
    """k_step's Y+ branch (X2H): with rel = X Y - m Y, the Phi products follow from S1 = <Y, XY>,
    S2 = |XY|^2, S3 = <XY, X^2 Y>: <Y, X rel> + <rel, XY> = 2 (S2 - m S1), <rel, X rel> = S3 - 2 m S2 + m^2 S1;
    and X rel = X^2 Y - m XY (IHO/simulation_i.cpp:301-333 computes X rel directly)."""
    rng = np.random.default_rng(5)
    ops = R.fock_ops(60, pi, inverted=True)
    x = ops["x"]
    y = rng.normal(size=61) + 1j * rng.normal(size=61)
    y /= np.linalg.norm(y)
    xy = x @ y
    m = np.vdot(y, xy).real
    rel = xy - m * y
    s1, s2, s3 = np.vdot(y, xy).real, np.vdot(xy, xy).real, np.vdot(xy, x @ xy).real
    direct0 = np.vdot(y, x @ rel).real + np.vdot(rel, xy).real
    direct1 = np.vdot(rel, x @ rel).real
    assert abs(direct0 - 2 * (s2 - m * s1)) < 1e-13
    assert abs(direct1 - (s3 - 2 * m * s2 + m * m * s1)) < 1e-13
