"""Drop-in surface of the reference CPython extension `simulation` (one env, numpy state).

The reference builds one extension per physical system with compile-time macros (*/setupC.py) and
the drivers call (IHO/main_parallel.py:174-264, IQO/main_parallel.py:123-218):

    simulation = __import__('simulation')
    simulation.set_seed(seed)
    q, x_mean, Fail = simulation.step(state, time_step, force, gamma)   # state mutated in place
    simulation.x_expectation(state); simulation.get_moments(state, data); simulation.check_settings()

Here the compile-time parameters become arguments of `load()`, which returns a module-like object
with the same function names, signatures, return values and error behaviour; each call runs the HIP
kernels of libqcart (B = 1) and copies the numpy state to and from the device (pinned staging, one copy each way). This surface exists
for drop-in compatibility; the throughput path is core.Stepper / env.BatchedEnv.

Noise: set_seed(seed) starts the reference's stream — MT19937 seeded like vslNewStream(VSL_BRNG_MT19937,
seed), two Box-Muller normals per step (qc_set_seed_mt19937; MKL's uniform words bit for bit, its
normals to <= 1 ulp of MKL's CBWR=COMPATIBLE path, tests/test_mkl_fixtures.py). Before the first
set_seed the module, like the reference's, has no seeded stream; here it draws from seed 0's.
load(..., noise="philox") selects the counter-based Philox stream instead.
"""
from __future__ import annotations

import ctypes
import sys
import types
from math import pi

import numpy as np

from . import _lib
from . import config as cfg

_MODULES: dict = {}
_MAX_STEPS = 10   # physics steps per drop-in call: step 1, simulate_10_steps 10


def _check_state(state, N):
    if not isinstance(state, np.ndarray):
        raise TypeError("The input object cannot be identified as a Numpy array")
    if state.ndim != 1:
        raise ValueError("The input array is not one-dimensional")
    if state.shape[0] != N:
        raise ValueError("The input array does not match the required size " + str(N))
    if state.dtype != np.complex128:
        raise ValueError("The input array does not match the required datatype: Complex128")


class _Simulation:
    """One compiled-parameter set of the reference module (see load())."""

    def __init__(self, physics: cfg.Physics, device: int = 0, noise: str = "mt19937"):
        import torch

        from .core import Stepper
        if noise not in ("mt19937", "philox"):
            raise ValueError("noise must be 'mt19937' or 'philox'")
        if physics.precision != 0:
            raise ValueError("the drop-in computes in fp64 like the reference (precision=0)")
        self._torch = torch
        self.physics = physics
        self._noise = noise
        self._st = Stepper(physics, 1, device, seed=0)
        if noise == "mt19937":
            self._st.set_seed_mt19937(0)
        self._dev = self._st.device
        self._dt, self._gamma = physics.dt, physics.gamma
        self.N = N = self._st.N
        # one device block per module and its pinned host mirror: psi (2N doubles) | q [10] | x_mean [10] |
        # Fail (int32 in one double slot). A call copies the state in through the pinned mirror and brings
        # psi, q, x_mean and Fail back in ONE asynchronous copy, with no per-call allocation
        self._blk_len = 2 * N + 2 * _MAX_STEPS + 1
        self._dblk = torch.zeros(self._blk_len, dtype=torch.float64, device=self._dev)
        self._hblk = torch.zeros(self._blk_len, dtype=torch.float64, pin_memory=True)
        self._hnp = self._hblk.numpy()
        self._hpsi_np = self._hnp[:2 * N].view(np.complex128)
        self._psi = self._dblk[:2 * N].view(torch.complex128).view(1, N)
        self._hpsi = self._hblk[:2 * N].view(torch.complex128).view(1, N)
        base = self._dblk.data_ptr()
        self._q_ptr = ctypes.c_void_p(base + 8 * 2 * N)
        self._xm_ptr = ctypes.c_void_p(base + 8 * (2 * N + _MAX_STEPS))
        self._fail_ptr = ctypes.c_void_p(base + 8 * (2 * N + 2 * _MAX_STEPS))
        self._psi_ptr = ctypes.c_void_p(base)

    # set_seed(int): IHO/simulation_i.cpp:574-579
    def set_seed(self, seed):
        if not isinstance(seed, (int, np.integer)):
            raise TypeError("seed must be an int")
        if self._noise == "mt19937":
            # PyArg "i" then vslNewStream(..., MKL_UINT seed): the int's low 32 bits
            self._st.set_seed_mt19937(int(seed) & 0xFFFFFFFF)
        else:
            self._st.set_seed(int(seed) & 0xFFFFFFFFFFFFFFFF)
        return None

    # check_settings(): IHO/simulation_i.cpp:581-583 -> (n_max, omega); QO:652-654 -> (x_n, h, lambda, mass, moment)
    def check_settings(self):
        p = self.physics
        if p.fock:
            return (p.n_max, p.omega)
        return (self.N, p.grid_size, p.lambda_, p.mass, p.moment_order)

    def _sync_dynamics(self, dt, gamma):
        if dt != self._dt or gamma != self._gamma:
            self._st.set_dynamics(float(dt), float(gamma))
            self._dt, self._gamma = dt, gamma

    def _slot(self, force):
        p = self.physics
        half = p.n_actions // 2
        spacing = p.f_max / half
        a = round(force / spacing)
        if -half <= a <= half and (a * spacing) == force:
            return a + half
        return self._st.add_force(float(force))

    def _run(self, state, dt, force, gamma, n, final_fail: bool):
        """n physics steps on the device; returns (q, x_mean, Fail) of the call (last step's q / x_mean;
        Fail = any step's boundary test (step) or the final state's (simulate_10_steps)). One host->device
        copy of the state and ONE device->host copy of state + the three scalars per call."""
        N = self.N
        _check_state(state, N)
        self._sync_dynamics(float(dt), float(gamma))
        slot = self._slot(float(force))
        st, lib = self._st, _lib.lib()
        np.copyto(self._hpsi_np, state)
        self._psi.copy_(self._hpsi, non_blocking=True)
        st._bind_stream()
        _lib.check(lib.qc_step(st._h, self._psi_ptr, None, int(slot), int(n), None, None, self._q_ptr,
                               self._xm_ptr, self._fail_ptr, None, None), st._h)
        if final_fail:
            _lib.check(lib.qc_boundary_fail(st._h, self._psi_ptr, self._fail_ptr), st._h)
        self._hblk.copy_(self._dblk, non_blocking=True)
        self._torch.cuda.current_stream(self._dev).synchronize()
        h = self._hnp
        state[:] = self._hpsi_np
        fail = int(h[2 * N + 2 * _MAX_STEPS:2 * N + 2 * _MAX_STEPS + 1].view(np.int32)[0])
        return float(h[2 * N + n - 1]), float(h[2 * N + _MAX_STEPS + n - 1]), int(fail > 0)

    # step(state, dt, force, gamma) -> (q, x_mean, Fail): IHO/simulation_i.cpp:358-389
    def step(self, state, dt, force, gamma):
        return self._run(state, dt, force, gamma, 1, False)

    # simulate_10_steps: IHO/simulation_i.cpp:391-421 (last step's q, x_mean; Fail of the final state)
    def simulate_10_steps(self, state, dt, force, gamma):
        return self._run(state, dt, force, gamma, 10, True)

    # x_expectation(state): IHO/simulation_i.cpp:204-215, QO/simulation_quart.cpp:244-258
    def x_expectation(self, state):
        _check_state(state, self.N)
        self._psi.copy_(self._torch.from_numpy(state).view(1, -1))
        return float(self._st.x_expectation(self._psi)[0])

    # get_moments(state, data): QO/simulation_quart.cpp:363-388 (grid families only in the reference)
    def get_moments(self, state, data):
        _check_state(state, self.N)
        n = self._st.n_obs
        if not isinstance(data, np.ndarray) or data.ndim != 1:
            raise ValueError("The moment data array is not one-dimensional")
        if data.shape[0] != n:
            raise ValueError("The moment data array does not match the required size " + str(n))
        if data.dtype != np.float64:
            raise ValueError("The moment data array does not match the required datatype: Float64")
        self._psi.copy_(self._torch.from_numpy(state).view(1, -1))
        data[:] = self._st.moments(self._psi)[0].cpu().numpy()
        return None


def load(family: int | str = cfg.IHO, device: int = 0, noise: str = "mt19937", **params) -> types.ModuleType:
    """Return a module-like object equivalent to the reference's compiled `simulation` extension.

    family: 0/'harmonic', 1/'inverted_harmonic', 2/'quartic', 3/'inverted_quartic'; params are the
    setupC.py macros (n_max, omega / x_max, grid_size, lambda_, mass, moment_order) and optionally
    gamma, time_steps, f_max, a_mode (defaults: the drivers' values, config.DEFAULTS). noise: 'mt19937'
    (the reference's stream, default) or 'philox'."""
    if isinstance(family, str):
        family = {v: k for k, v in cfg.FAMILY_NAMES.items()}[family]
    phys = cfg.DEFAULTS[family].with_(**params)
    key = (device, noise, tuple(sorted(phys.asdict().items())))
    if key not in _MODULES:
        sim = _Simulation(phys, device, noise)
        mod = types.ModuleType("simulation", "MI355X-native drop-in for the reference `simulation` module")
        for name in ("step", "simulate_10_steps", "set_seed", "check_settings", "x_expectation"):
            setattr(mod, name, getattr(sim, name))
        if not phys.fock:
            mod.get_moments = sim.get_moments
        mod._impl = sim
        _MODULES[key] = mod
    return _MODULES[key]


def install(family: int | str = cfg.IHO, device: int = 0, noise: str = "mt19937", **params) -> types.ModuleType:
    """Register the drop-in as `simulation` in sys.modules, so the reference drivers'
    `__import__('simulation')` resolves to it."""
    mod = load(family, device, noise, **params)
    sys.modules["simulation"] = mod
    return mod


__all__ = ["load", "install", "pi"]
