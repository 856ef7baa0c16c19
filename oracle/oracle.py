"""ctypes wrapper over the CPU restatement (oracle/qcart_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, as the checker. The product path (deepreinforcementlearningcontrolofquantumcartpoles_amd)
never imports this module. Parity vs the reference binary is UNPINNED (see qcart_oracle.h).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from math import pi

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "libqcart_oracle.so")

HO, IHO, QO, IQO = 0, 1, 2, 3


class QoParams(ctypes.Structure):
    _fields_ = [
        ("family", ctypes.c_int32),
        ("n_max", ctypes.c_int32),
        ("omega", ctypes.c_double),
        ("x_max", ctypes.c_double),
        ("grid_size", ctypes.c_double),
        ("lambda_", ctypes.c_double),
        ("mass", ctypes.c_double),
        ("moment_order", ctypes.c_int32),
        ("a_mode", ctypes.c_int32),
    ]


def build(force: bool = False) -> str:
    src = os.path.join(_HERE, "qcart_oracle.c")
    if force or not os.path.exists(_SO) or os.path.getmtime(_SO) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _SO


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        P = ctypes.POINTER
        d, i32, i64, u64 = ctypes.c_double, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64
        vp = ctypes.c_void_p
        L.qo_create.restype = vp
        L.qo_create.argtypes = [P(QoParams)]
        L.qo_destroy.argtypes = [vp]
        L.qo_dim.argtypes = [vp]
        L.qo_n_obs.argtypes = [vp]
        L.qo_make_tab.restype = vp
        L.qo_make_tab.argtypes = [vp, d, d, P(ctypes.c_int)]
        L.qo_free_tab.argtypes = [vp]
        L.qo_step.argtypes = [vp, vp, vp, d, d, d, vp, P(d), P(d), P(ctypes.c_int)]
        L.qo_x_expectation.restype = d
        L.qo_x_expectation.argtypes = [vp, vp]
        L.qo_moments.argtypes = [vp, vp, vp]
        L.qo_outside_prob.restype = d
        L.qo_outside_prob.argtypes = [vp, vp, d]
        L.qo_boundary_fail.argtypes = [vp, vp]
        L.qo_energy.restype = d
        L.qo_energy.argtypes = [vp, vp]
        L.qo_phonon.restype = d
        L.qo_phonon.argtypes = [vp, vp]
        L.qo_dense_h.argtypes = [vp, vp]
        L.qo_dense_x.argtypes = [vp, vp]
        L.qo_tab_ldab.argtypes = [vp]
        L.qo_tab_export.argtypes = [vp, vp, vp, vp]
        L.qo_philox4x32_10.argtypes = [vp, vp, vp]
        L.qo_normals.argtypes = [u64, u64, u64, vp]
        L.qo_term7.argtypes = [vp, vp, vp, vp]
        L.qo_tab_solve.argtypes = [vp, vp]
        L.qo_grid_p_apply.argtypes = [vp, vp, d, vp]
        L.qo_mt_seed.argtypes = [ctypes.c_uint32, vp]
        L.qo_mt_next.argtypes = [vp]
        L.qo_mt_next.restype = ctypes.c_uint32
        L.qo_mt_normals.argtypes = [vp, i64, vp]
        L.qo_fock_random_state.argtypes = [vp, u64, u64, ctypes.c_int, vp]
        L.qo_gaussian_packet.argtypes = [vp, d, d, d, vp]
        L.qo_run_batch.argtypes = [vp, vp, i64, vp, d, ctypes.c_int, d, d, u64, i64, u64, vp, vp, vp,
                                   ctypes.c_int]
        L.qo_run_batch_noise.argtypes = [vp, vp, i64, vp, d, ctypes.c_int, d, d, vp, vp, vp, vp,
                                         ctypes.c_int]
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


class OracleSystem:
    """One compiled-parameter set of the reference `simulation` module, restated on the CPU."""

    def __init__(self, family: int, n_max: int = 0, omega: float = pi, x_max: float = 0.0,
                 grid_size: float = 0.0, lambda_: float = 0.0, mass: float = 0.0,
                 moment_order: int = 5, a_mode: int = 0):
        self.params = QoParams(family, n_max, omega, x_max, grid_size, lambda_, mass, moment_order,
                               a_mode)
        self.family = family
        self._h = lib().qo_create(ctypes.byref(self.params))
        if not self._h:
            raise ValueError("invalid oracle parameters")
        self.N = lib().qo_dim(self._h)
        self.n_obs = lib().qo_n_obs(self._h)
        self._tabs: dict = {}

    def __del__(self):
        try:
            for t in self._tabs.values():
                lib().qo_free_tab(t)
            if self._h:
                lib().qo_destroy(self._h)
        except Exception:
            pass

    def tab(self, dt: float, force: float):
        key = (float(dt), float(force))
        if key not in self._tabs:
            nsw = ctypes.c_int(0)
            t = lib().qo_make_tab(self._h, dt, force, ctypes.byref(nsw))
            if not t:
                raise RuntimeError("band LU failed (singular)")
            self._tabs[key] = t
            self._tabs[("nswap",) + key] = nsw.value
        return self._tabs[key]

    def n_swaps(self, dt: float, force: float) -> int:
        self.tab(dt, force)
        return self._tabs[("nswap", float(dt), float(force))]

    def step(self, psi: np.ndarray, dt: float, force: float, gamma: float, r):
        assert psi.dtype == np.complex128 and psi.shape == (self.N,) and psi.flags.c_contiguous
        rr = np.ascontiguousarray(np.asarray(r, dtype=np.float64))
        q, xm, f = ctypes.c_double(), ctypes.c_double(), ctypes.c_int()
        lib().qo_step(self._h, self.tab(dt, force), _ptr(psi), dt, force, gamma, _ptr(rr),
                      ctypes.byref(q), ctypes.byref(xm), ctypes.byref(f))
        return q.value, xm.value, f.value

    def x_expectation(self, psi):
        return lib().qo_x_expectation(self._h, _ptr(np.ascontiguousarray(psi)))

    def moments(self, psi):
        out = np.zeros(self.n_obs, dtype=np.float64)
        lib().qo_moments(self._h, _ptr(np.ascontiguousarray(psi)), _ptr(out))
        return out

    def outside_prob(self, psi, xth):
        return lib().qo_outside_prob(self._h, _ptr(np.ascontiguousarray(psi)), xth)

    def boundary_fail(self, psi):
        return lib().qo_boundary_fail(self._h, _ptr(np.ascontiguousarray(psi)))

    def energy(self, psi):
        return lib().qo_energy(self._h, _ptr(np.ascontiguousarray(psi)))

    def phonon(self, psi):
        return lib().qo_phonon(self._h, _ptr(np.ascontiguousarray(psi)))

    def dense_h(self):
        out = np.zeros((self.N, self.N))
        lib().qo_dense_h(self._h, _ptr(out))
        return out

    def dense_x(self):
        out = np.zeros((self.N, self.N))
        lib().qo_dense_x(self._h, _ptr(out))
        return out

    def tab_export(self, dt, force):
        t = self.tab(dt, force)
        ldab = lib().qo_tab_ldab(t)
        kl = {HO: 1, IHO: 2}.get(self.family, 4)
        ab = np.zeros((self.N, ldab), dtype=np.complex128)   # column-major AB: ab[col, row]
        ipiv = np.zeros(self.N, dtype=np.int32)
        A = np.zeros((2 * 5 * kl + 1, self.N), dtype=np.complex128)
        lib().qo_tab_export(t, _ptr(ab), _ptr(ipiv), _ptr(A))
        return ab, ipiv, A

    def term7(self, dt, force, v):
        y = np.zeros(self.N, dtype=np.complex128)
        lib().qo_term7(self._h, self.tab(dt, force), _ptr(np.ascontiguousarray(v, np.complex128)), _ptr(y))
        return y

    def tab_solve(self, dt, force, b):
        x = np.ascontiguousarray(b, np.complex128).copy()
        lib().qo_tab_solve(self.tab(dt, force), _ptr(x))
        return x

    def grid_p_apply(self, v, pbar):
        y = np.zeros(self.N, dtype=np.complex128)
        lib().qo_grid_p_apply(self._h, _ptr(np.ascontiguousarray(v, np.complex128)), pbar, _ptr(y))
        return y

    def fock_random_state(self, seed, env_id, levels=16):
        psi = np.zeros(self.N, dtype=np.complex128)
        lib().qo_fock_random_state(self._h, seed, env_id, levels, _ptr(psi))
        return psi

    def gaussian_packet(self, wavenumber, mean, std):
        psi = np.zeros(self.N, dtype=np.complex128)
        lib().qo_gaussian_packet(self._h, wavenumber, mean, std, _ptr(psi))
        return psi

    def run_batch(self, psi: np.ndarray, actions: np.ndarray, f_max: float, n_steps: int, dt: float,
                  gamma: float, seed: int = 0, env_offset: int = 0, step0: int = 0,
                  noise: np.ndarray | None = None, want_q: bool = False, n_threads: int = 0):
        """Advance psi[B, N] (in place) n_steps with per-env discrete actions."""
        assert psi.dtype == np.complex128 and psi.ndim == 2 and psi.shape[1] == self.N
        assert psi.flags.c_contiguous
        B = psi.shape[0]
        act = np.ascontiguousarray(actions, dtype=np.int32)
        fail = np.zeros(B, dtype=np.int32)
        q = np.zeros((n_steps, B)) if want_q else None
        xm = np.zeros((n_steps, B)) if want_q else None
        qp = _ptr(q) if want_q else None
        xp = _ptr(xm) if want_q else None
        if noise is None:
            rc = lib().qo_run_batch(self._h, _ptr(psi), B, _ptr(act), f_max, n_steps, dt, gamma, seed,
                                    env_offset, step0, _ptr(fail), qp, xp, n_threads)
        else:
            nz = np.ascontiguousarray(noise, dtype=np.float64)
            assert nz.shape == (n_steps, B, 2)
            rc = lib().qo_run_batch_noise(self._h, _ptr(psi), B, _ptr(act), f_max, n_steps, dt, gamma,
                                          _ptr(nz), _ptr(fail), qp, xp, n_threads)
        if rc != 0:
            raise RuntimeError(f"oracle run_batch failed rc={rc}")
        return fail, q, xm


def normals(seed: int, env_id: int, step: int):
    r = np.zeros(2)
    lib().qo_normals(seed, env_id, step, _ptr(r))
    return r


def philox(ctr, key):
    c = np.ascontiguousarray(ctr, dtype=np.uint32)
    k = np.ascontiguousarray(key, dtype=np.uint32)
    o = np.zeros(4, dtype=np.uint32)
    lib().qo_philox4x32_10(_ptr(c), _ptr(k), _ptr(o))
    return o


class MT19937:
    """The reference's noise stream restated (set_seed + vdRngGaussian BOXMULLER, IHO/simulation_i.cpp:
    574-579, :435): MT19937 seeded by init_by_array({seed}), normals sqrt(-2 ln u1) sin(2 pi u2)."""

    def __init__(self, seed: int):
        self.st = np.zeros(625, dtype=np.uint32)
        lib().qo_mt_seed(int(seed) & 0xFFFFFFFF, _ptr(self.st))

    def words(self, n: int) -> np.ndarray:
        return np.array([lib().qo_mt_next(_ptr(self.st)) for _ in range(n)], dtype=np.uint32)

    def normals(self, n: int) -> np.ndarray:
        out = np.zeros(n, dtype=np.float64)
        lib().qo_mt_normals(_ptr(self.st), n, _ptr(out))
        return out


def mt_noise(seeds, n_steps: int) -> np.ndarray:
    """[n_steps][B][2] normals of per-env MT19937 streams (the reference's 2 draws per step)."""
    return np.stack([MT19937(s).normals(2 * n_steps).reshape(n_steps, 2) for s in seeds], axis=1)
