"""Dense numpy restatements used to pin the C oracle (test infrastructure).

These follow the reference's own *Python* operator definitions (restated, not imported — importing
or running the reference is denied here):
  * Fock operators: IHO/main_parallel.py:53-79 (adjust_n_max), HO/main_parallel.py:73
  * Grid operators: QO/space_def.py:5-88 (set_global)
and Appendix A of SURVEY.md (the go_one_step scheme of IHO/simulation_i.cpp:432-489) as dense algebra.
"""
from __future__ import annotations

from math import pi, sqrt

import numpy as np

HO, IHO, QO, IQO = 0, 1, 2, 3


def fock_ops(n_max: int, omega: float = pi, inverted: bool = True):
    """adjust_n_max(): a, a+, x, p, x^2, Re(p^2), xp+px, H (IHO/main_parallel.py:53-79)."""
    sqrt_n = np.array([sqrt(i) for i in range(1, n_max + 1)])
    ann = np.diag(sqrt_n, k=1)
    cre = np.diag(sqrt_n, k=-1)
    x = sqrt(1 / 2) * (cre + ann)
    p = 1.0j * sqrt(1 / 2) * (cre - ann)
    x2 = x @ x
    p2 = np.real(p @ p)
    xppx = x @ p + p @ x
    if inverted:
        H = -1 / 2 * omega * (cre @ cre + ann @ ann)
    else:
        H = omega * np.diag(1 / 2 + np.arange(n_max + 1, dtype=np.float64))
    return dict(x=x, p=p, x2=x2, p2=p2, xppx=xppx, H=H)


def grid_ops(x_max: float, grid_size: float, lambda_: float, mass: float):
    """set_global() of QO/space_def.py:5-88, with x_n = 2*int(x_max/h + 0.5) + 1 (C convention)."""
    half = int(x_max / grid_size + 0.5)
    n = 2 * half + 1
    x = grid_size * (np.arange(n) - half)
    di1, di2 = np.diag_indices(n)
    dx = np.zeros((n, n))
    dx[(di1[:-1], di2[1:])] = 672 / 840
    dx[(di1[1:], di2[:-1])] = -672 / 840
    dx[(di1[:-2], di2[2:])] = -168 / 840
    dx[(di1[2:], di2[:-2])] = 168 / 840
    dx[(di1[:-3], di2[3:])] = 32 / 840
    dx[(di1[3:], di2[:-3])] = -32 / 840
    dx[(di1[:-4], di2[4:])] = -3 / 840
    dx[(di1[4:], di2[:-4])] = 3 / 840
    dx /= grid_size
    d2 = np.zeros((n, n))
    d2[(di1, di2)] = -14350 / 5040
    for k, v in ((1, 8064), (2, -1008), (3, 128), (4, -9)):
        d2[(di1[:-k], di2[k:])] = v / 5040
        d2[(di1[k:], di2[:-k])] = v / 5040
    d2 /= grid_size ** 2
    p = -1.0j * dx
    H = np.diag(lambda_ * x ** 4) + (-d2) / (2.0 * mass)
    return dict(x=x, X=np.diag(x), dx=dx, p=p, H=H, d2=d2, n=n, h=grid_size)


def correction_A(HF: np.ndarray, dt: float) -> np.ndarray:
    """Hamiltonian_addup_factor (IHO/simulation_i.cpp:253-264)."""
    H2 = HF @ HF
    H3 = H2 @ HF
    H4 = H2 @ H2
    H5 = H2 @ H3
    return dt ** 3 / 12 * H2 - 1j * dt ** 4 / 24 * H3 - dt ** 5 / 80 * H4 + 1j * dt ** 6 / 360 * H5


def mirror(A: np.ndarray, hermitian: bool) -> np.ndarray:
    """MKL sparse mv with FILL_MODE_UPPER: triu(A) + triu(A,1)^T (SYMMETRIC) or ^H (HERMITIAN)."""
    U = np.triu(A)
    L = np.triu(A, 1).T
    return U + (np.conj(L) if hermitian else L)


def dense_step(psi, H, X, F, c, gamma, dt, r, w, A_eff):
    """SURVEY.md Appendix A, dense. Returns (psi_new, q, x_mean)."""
    HF = H - c * F * X
    beta = sqrt(gamma / 2)
    dW = r[0] * sqrt(dt)
    dZ = sqrt(dt) * dt * 0.5 * (r[0] + r[1] / sqrt(3.0))

    def mean(v):
        return np.real(np.vdot(v, X @ v)) * w

    xm = mean(psi)
    q = xm + dW / sqrt(2 * gamma) / dt if gamma > 0 else xm
    rel = X @ psi - xm * psi
    D1 = -1j * (HF @ psi) - gamma / 4 * (X @ rel - xm * rel)
    D2 = beta * rel
    Yp = psi + dt * D1 + sqrt(dt) * D2
    Ym = psi + dt * D1 - sqrt(dt) * D2

    def parts(Y):
        ym = mean(Y)
        rl = X @ Y - ym * Y
        return -1j * (HF @ Y), -gamma / 4 * (X @ rl - ym * rl), beta * rl

    Ip, Rp, D2p = parts(Yp)
    Im, Rm, D2m = parts(Ym)
    dIm = Ip - Im
    Php = Yp + sqrt(dt) * D2p
    Phm = Yp - sqrt(dt) * D2p

    def d2fresh(P):
        pm = mean(P)
        return beta * (X @ P - pm * P)

    D2Pp, D2Pm = d2fresh(Php), d2fresh(Phm)
    sdt = sqrt(dt)
    rhs = (psi + D2 * dW + 0.5 / sdt * dZ * (dIm + Rp - Rm) + 0.25 * dt * (Rp + 2 * D1 + Rm)
           + 0.25 / sdt * (dW * dW - dt) * (D2p - D2m) + 0.5 / dt * (dW * dt - dZ) * (D2p + D2m - 2 * D2)
           + 0.25 / dt * (dW * dW / 3 - dt) * dW * (D2Pp - D2Pm - D2p + D2m) - 0.25 * sdt * dW * dIm
           + A_eff @ D1)
    M = np.eye(len(psi)) + 1j * dt / 2 * HF
    new = np.linalg.solve(M, rhs)
    new /= np.linalg.norm(new) * sqrt(w)
    return new, q, xm


def hermitian_p_grid(g):
    """p_hat under the HERMITIAN/UPPER mv descriptor with the C module's truncated Delta_1 loops
    (QO/simulation_quart.cpp:59-70): upper entry (r, r+d) exists iff r <= n-1-2d."""
    n = g["n"]
    h = g["h"]
    P = np.zeros((n, n), dtype=np.complex128)
    sd = {1: 672.0, 2: -168.0, 3: 32.0, 4: -3.0}
    for d, v in sd.items():
        for r in range(0, n - 2 * d):
            P[r, r + d] = -1j * (v / 840.0 / h)
            P[r + d, r] = np.conj(P[r, r + d])
    return P


def grid_moments_dense(psi, g, order=5):
    """compute_statistics (QO/simulation_quart.cpp:326-362) in dense numpy."""
    h = g["h"]
    P = hermitian_p_grid(g)
    xe = np.real(np.vdot(psi, g["x"] * psi)) * h
    pe = np.real(np.vdot(psi, P @ psi)) * h
    xr = g["x"] - xe
    Pr = P - pe * np.eye(g["n"])
    out = [xe, pe]
    for j in range(2, order + 1):
        for i in range(j + 1):
            v = psi.copy()
            for _ in range(i):
                v = Pr @ v
            v = xr ** (j - i) * v
            out.append(np.real(np.vdot(psi, v)) * h)
    return np.array(out)
