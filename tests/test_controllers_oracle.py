"""CPU checks of the controller oracle (oracle/controllers.py) against closed forms: coherent-state
and Gaussian-packet expectations, and the reference's rounding semantics (Python round(): ties to
even; clip to +-F_max)."""
from math import exp, pi, sqrt

import numpy as np
import pytest

from oracle import controllers as OC


def coherent(alpha, n_max):
    from math import factorial
    n = np.arange(n_max + 1)
    c = np.array([alpha ** k / sqrt(float(factorial(k))) for k in n], dtype=np.complex128)
    return c * exp(-abs(alpha) ** 2 / 2)


def test_fock_data_on_coherent_state():
    alpha = 0.7 - 0.4j
    psi = coherent(alpha, 60)
    d = OC.get_data_xp(psi, OC.fock_ops(60))
    # x = sqrt2 Re alpha, p = sqrt2 Im alpha, variances 1/2, covariance 0
    np.testing.assert_allclose(d, [sqrt(2) * alpha.real, sqrt(2) * alpha.imag, 0.5, 0.5, 0.0], atol=1e-6)


def test_fock_lqg_formula():
    alpha = 0.2 + 0.1j
    psi = coherent(alpha, 40)
    x, p = sqrt(2) * alpha.real, sqrt(2) * alpha.imag
    T, w = 1 / 18, pi
    F = -(x + p) * (1 + w * T + 0.5 * w * w * T * T) / (T + w * T * T / 2) / w
    a, f = OC.fock_lqg(psi, 1, pi, 18, 8.0)
    assert a == round(F / 0.8) + 10 and f == pytest.approx(round(F / 0.8) * 0.8)
    F_ho = -((x + p) + (p - x) * w * T) / T / w
    a, f = OC.fock_lqg(psi, 0, pi, 18, 5.0)
    assert a == round(F_ho / 0.5) + 10


def test_round_semantics():
    # ties to even (Python round), clipping at +-F_max
    assert OC._round_force(0.25, 5.0) == (10, 0.0)        # 0.5 -> 0
    assert OC._round_force(0.75, 5.0) == (12, 1.0)        # 1.5 -> 2
    assert OC._round_force(-0.75, 5.0) == (8, -1.0)
    assert OC._round_force(99.0, 8.0) == (20, 8.0)
    assert OC._round_force(-99.0, 8.0) == (0, -8.0)


def test_grid_expectations_gaussian_packet():
    g = OC.Grid(8.5, 171)
    mu, sg, k = 0.4, 0.9, 0.3
    x = g.x
    psi = np.exp(2.j * pi * (x - mu) * k) * np.exp(-(x - mu) ** 2 / (4 * sg * sg))
    psi /= np.linalg.norm(psi) * sqrt(g.grid_size)
    xe, pe, x2, x3, xpx = g.expectations(psi)
    p0 = 2 * pi * k
    assert xe == pytest.approx(mu, abs=1e-10)
    assert pe == pytest.approx(p0, rel=1e-6)
    assert x2 == pytest.approx(mu * mu + sg * sg, rel=1e-9)
    assert x3 == pytest.approx(mu ** 3 + 3 * mu * sg * sg, rel=1e-9)
    assert xpx == pytest.approx(p0 * (mu * mu + sg * sg), rel=1e-6)


def test_grid_controllers_closed_form():
    g = OC.Grid(8.5, 171)
    lam, m, n_con = 0.04 * pi, 1 / pi, 18
    mu, sg, k = -0.5, 1.1, 0.1
    x = g.x
    psi = np.exp(2.j * pi * (x - mu) * k) * np.exp(-(x - mu) ** 2 / (4 * sg * sg))
    psi /= np.linalg.norm(psi) * sqrt(g.grid_size)
    xe, pe, x2, x3, xpx = g.expectations(psi)
    T = 1 / n_con
    pp = pe - 4 * lam * x3 * T - T * T * 6 * lam * xpx / m
    assert OC.grid_force(g, psi, "damping", 0.5, lam, m, n_con) == pytest.approx(-pp / T * 0.5)
    tp = -sqrt(2 * m * (6 * lam * (x2 - xe * xe) + lam * xe * xe)) * xe
    assert OC.grid_force(g, psi, "semiclassical", 0, lam, m, n_con) == pytest.approx((tp - pe) / T)
    with pytest.raises(ValueError):   # the reference's math domain error for lambda < 0
        OC.grid_force(g, psi, "semiclassical", 0, -lam, m, n_con)
