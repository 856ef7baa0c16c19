"""numpy restatement of the reference's analytic baseline controllers.

TEST INFRASTRUCTURE ONLY: the checker of qc_control (csrc/qcart_kernels.hpp k_control), imported by
tests/ only. Pure numpy on dense operators, for small N.

Follows, in the reference tree `implementation codes/`:
  harmonic oscillator/main_parallel.py:192-203            HO args.LQG branch of call_force
  inverted harmonic oscillator/main_parallel.py:194-206   IHO args.LQG branch of call_force
  inverted harmonic oscillator/main_parallel.py:53-71,92-99,129-131  Fock operators and get_data_xp
  quartic oscillator/controllers.py:7-29                  steepest_descent / LinearQuadratic / Gaussian_approx
  quartic oscillator/main_parallel.py:165-181             analytic_controls: F / pi, clip, round
  quartic oscillator/space_def.py:5-21,59                 grid x, grid_size, p_hat = -i Delta_1
Numeric types: the Fock branch reads x, p from the float32 network input; `x + p` is a float32 sum and
the remaining arithmetic is fp64 (numpy 1.x promotes a float32 scalar times a Python float to float64;
numpy >= 2 would keep float32, so the promotion is written out explicitly here).
Parity anchor: no reference outputs exist for the controllers; this restatement is the
formula text itself, checked in tests/test_controllers.py against hand-evaluated states.
"""
from __future__ import annotations

from math import pi, sqrt

import numpy as np


def fock_ops(n_max: int):
    """x_hat, p_hat, x_hat_2, p_hat_2, xp_px_hat (IHO/main_parallel.py:53-71) as dense arrays."""
    sq = np.sqrt(np.arange(1, n_max + 1, dtype=np.float64))
    ann = np.diag(sq, k=1)
    cre = np.diag(sq, k=-1)
    x = sqrt(1 / 2) * (cre + ann)
    p = 1.0j * sqrt(1 / 2) * (cre - ann)
    return x, p, x @ x, np.real(p @ p), x @ p + p @ x


def get_data_xp(state, ops) -> np.ndarray:
    x_hat, p_hat, x2, p2, xp = ops
    ex = lambda op: np.real(np.conj(state).dot(op.dot(state)))  # noqa: E731
    xe, pe = ex(x_hat), ex(p_hat)
    return np.array([xe, pe, ex(x2) - xe ** 2, ex(p2) - pe ** 2, ex(xp) / 2 - xe * pe]).astype(np.float32)


def _round_force(force: float, f_max: float, half: int = 10):
    """clip + Python round() to the action grid (QO/main_parallel.py:175-181, IHO:198-205)."""
    force_max = round(2 * half - half) * (f_max / half)   # net.convert_to_force(2 * no_action_choice)
    force = min(force, force_max)
    force = max(force, -force_max)
    force = round(force / (force_max / half))
    force = float(force * (force_max / half))
    return round(force / (force_max / half)) + half, force


def fock_lqg(state, family: int, omega: float, n_con: int, f_max: float, input_scaling: float = 1.0, ops=None):
    """HO (family 0) / IHO (family 1) args.LQG control from data = get_data_xp(state) * input_scaling."""
    if ops is None:
        ops = fock_ops(state.size - 1)
    data = get_data_xp(state, ops) * np.float32(input_scaling)
    x, p = np.float32(data[0]), np.float32(data[1])
    dt = 1. / n_con
    s = float(np.float32(x + p))
    if family == 1:
        F = -s * (1 + omega * dt + 0.5 * omega * omega * dt * dt) / (dt + omega * dt * dt / 2)
    else:
        F = - (s + float(np.float32(p - x)) * omega * dt) / dt
    return _round_force(F / omega, f_max)


class Grid:
    """space_def.set_global (QO/space_def.py:5-21,59) for x_max, x_n."""

    def __init__(self, x_max: float, x_n: int):
        n = x_n - 1
        self.grid_size = x_max * 2 / n
        self.x = np.linspace(-x_max, x_max, n + 1, dtype=np.float64)
        d = np.zeros((n + 1, n + 1))
        i1, i2 = np.diag_indices(n + 1)
        for k, c in ((1, 672 / 840), (2, -168 / 840), (3, 32 / 840), (4, -3 / 840)):
            d[(i1[:-k], i2[k:])] = c
            d[(i1[k:], i2[:-k])] = -c
        d /= self.grid_size
        self.p_hat = -1.j * d

    def expectations(self, state):
        h, x = self.grid_size, self.x
        xe = np.real(np.conj(state).dot(x * state)) * h
        pe = np.real(np.conj(state).dot(self.p_hat.dot(state))) * h
        x2 = np.real(np.conj(state).dot(x * x * state)) * h
        x3 = np.real(np.conj(state).dot(x ** 3 * state)) * h
        xpx = np.real(np.conj(state).dot(x * self.p_hat.dot(x * state))) * h
        return xe, pe, x2, x3, xpx


def grid_force(grid: Grid, state, strategy: str, con_parameter: float, lambda_: float, mass: float,
               n_con: int):
    """controllers.py:7-29 with control_time = 1 / controls_per_unit_time; returns F (before / pi)."""
    T = 1. / n_con
    xe, pe, x2, x3, xpx = grid.expectations(state)
    if strategy == "damping":
        pp = pe - 4. * lambda_ * x3 * T - T ** 2 * 2. * lambda_ * 3. * xpx / mass
        return -pp / T * con_parameter
    if strategy == "LQG":
        k = lambda_ * con_parameter
        xq = xe + pe / mass * T - T ** 2 * 2. * lambda_ * x3 / mass
        pq = pe - 4. * lambda_ * x3 * T - T ** 2 * 2. * lambda_ * 3. * xpx / mass
        return -(sqrt(k * mass) * xq + pq) / T
    var = x2 - xe ** 2
    tp = -sqrt(2 * mass * (6 * lambda_ * var + lambda_ * xe ** 2)) * xe
    return (tp - pe) / T


def grid_control(grid: Grid, state, strategy: str, con_parameter: float, lambda_: float, mass: float,
                 n_con: int, f_max: float):
    """analytic_controls (QO/main_parallel.py:165-181): (action, force)."""
    F = grid_force(grid, state, strategy, con_parameter, lambda_, mass, n_con)
    return _round_force(F / pi, f_max)
