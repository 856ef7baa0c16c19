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

The reference's process model — 30-40 actor processes, each with its own module stepping one env
(IHO/main_parallel.py:345-359) — runs through a step server: one process owns the GPU (StepServer / serve(),
qc_server_* in libqcart) and each actor calls load(..., server="/name") (or install(...)), whose functions post
requests through shared memory (libqcart_client.so, plain C: the actor process never creates a HIP context) and
are served for every pending actor in one batched launch per tick. Same names, arguments, return values, errors
and per-env MT19937 stream as the module above.
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

    # Hamiltonian_dot_psi(state): IHO/simulation_i.cpp:585-601, HO/simulation.cpp:566-582 — state <- H state in
    # place with the force-free Hamiltonian (mkl_sparse_z_mv of harmonic_Hamil); returns 0.0 like the reference
    def Hamiltonian_dot_psi(self, state):
        _check_state(state, self.N)
        self._psi.copy_(self._torch.from_numpy(state).view(1, -1))
        self._st.hamiltonian_dot_psi(self._psi)
        state[:] = self._psi[0].cpu().numpy()
        return 0.0

    # solve_ab(state): IHO/simulation_i.cpp:603-616, HO/simulation.cpp:584-598 — not reproduced: the IHO module
    # calls LAPACKE_zgbtrs with kl = ku = 1 on its kl = ku = 2 factorisation (a different, ill-defined operator) and
    # no driver calls it
    def solve_ab(self, state):
        _check_state(state, self.N)
        raise NotImplementedError("solve_ab is not reproduced (a debugging entry point of the reference modules that "
                                  "no driver calls; the IHO module's zgbtrs call uses the wrong band widths)")

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


# ---------------------------------------------------------------------------- step server (many actor processes)
_CLIENT_LIB = None


def _client_lib():
    """libqcart_client.so (include/qcart_client.h): plain C, no HIP — loading it never touches the GPU."""
    global _CLIENT_LIB
    if _CLIENT_LIB is None:
        import os
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libqcart_client.so")
        if not os.path.exists(path):
            raise ImportError(f"{path} not built: run `make`")
        L = ctypes.CDLL(path)
        vp, d, i32, P = ctypes.c_void_p, ctypes.c_double, ctypes.c_int32, ctypes.POINTER
        L.qcc_open.argtypes = [ctypes.c_char_p, P(vp)]
        L.qcc_close.argtypes = [vp]
        L.qcc_close.restype = None
        L.qcc_last_error.argtypes = [vp]
        L.qcc_last_error.restype = ctypes.c_char_p
        for f in ("qcc_dim", "qcc_n_obs", "qcc_family", "qcc_slot"):
            getattr(L, f).argtypes = [vp]
        L.qcc_settings.argtypes = [vp, vp]
        L.qcc_step.argtypes = [vp, vp, i32, d, d, d, P(d), P(d), P(i32)]
        L.qcc_set_seed.argtypes = [vp, ctypes.c_uint32]
        L.qcc_x_expectation.argtypes = [vp, vp, P(d)]
        L.qcc_moments.argtypes = [vp, vp, vp]
        L.qcc_hamiltonian_dot_psi.argtypes = [vp, vp]
        _CLIENT_LIB = L
    return _CLIENT_LIB


class _ServedSimulation:
    """One actor's `simulation` module served by a StepServer (one slot = one env of the server's batch)."""

    def __init__(self, physics: cfg.Physics, server: str):
        L = _client_lib()
        c = ctypes.c_void_p()
        rc = L.qcc_open(server.encode(), ctypes.byref(c))
        if rc != 0:
            raise RuntimeError("Initialization Failure: " + (L.qcc_last_error(None) or b"").decode())
        self._L, self._c = L, c
        self.physics = physics
        self.N = L.qcc_dim(c)
        self.n_obs = L.qcc_n_obs(c)
        st = np.zeros(9)
        L.qcc_settings(c, st.ctypes.data)
        fam = L.qcc_family(c)
        # the drivers' compile check (check_C_module_and_compile, IHO/main_parallel.py:564-583): the server's
        # module must carry this actor's parameters
        want = (physics.n_max, physics.omega) if physics.fock else (physics.x_max, physics.grid_size, physics.lambda_,
                                                                     physics.mass, physics.moment_order)
        have = (int(st[0]), st[1]) if physics.fock else (st[2], st[3], st[4], st[5], int(st[6]))
        if fam != physics.family or want != have:
            self.close()
            raise RuntimeError(f"step server {server} serves family {fam} {have}, not {physics.family} {want}")
        self._q, self._xm, self._f = ctypes.c_double(), ctypes.c_double(), ctypes.c_int32()
        self._v = ctypes.c_double()

    def close(self):
        if getattr(self, "_c", None):
            self._L.qcc_close(self._c)
            self._c = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != 0:
            msg = (self._L.qcc_last_error(self._c) or b"").decode()
            raise RuntimeError(f"step server: {msg} ({rc})")

    def set_seed(self, seed):
        if not isinstance(seed, (int, np.integer)):
            raise TypeError("seed must be an int")
        self._check(self._L.qcc_set_seed(self._c, int(seed) & 0xFFFFFFFF))

    def check_settings(self):
        p = self.physics
        return (p.n_max, p.omega) if p.fock else (self.N, p.grid_size, p.lambda_, p.mass, p.moment_order)

    def _run(self, state, dt, force, gamma, n):
        _check_state(state, self.N)
        if not state.flags.c_contiguous or not state.flags.writeable:
            raise ValueError("The input array is not a writeable contiguous array")
        self._check(self._L.qcc_step(self._c, state.ctypes.data, n, float(dt), float(force), float(gamma),
                                     ctypes.byref(self._q), ctypes.byref(self._xm), ctypes.byref(self._f)))
        return self._q.value, self._xm.value, int(self._f.value)

    def step(self, state, dt, force, gamma):
        return self._run(state, dt, force, gamma, 1)

    def simulate_10_steps(self, state, dt, force, gamma):
        return self._run(state, dt, force, gamma, 10)

    def x_expectation(self, state):
        _check_state(state, self.N)
        st = np.ascontiguousarray(state)
        self._check(self._L.qcc_x_expectation(self._c, st.ctypes.data, ctypes.byref(self._v)))
        return self._v.value

    # Hamiltonian_dot_psi(state) (Fock modules, IHO/simulation_i.cpp:585-601): served on the server's batch
    def Hamiltonian_dot_psi(self, state):
        _check_state(state, self.N)
        if not state.flags.c_contiguous or not state.flags.writeable:
            raise ValueError("The input array is not a writeable contiguous array")
        self._check(self._L.qcc_hamiltonian_dot_psi(self._c, state.ctypes.data))
        return 0.0

    solve_ab = _Simulation.solve_ab

    def get_moments(self, state, data):
        _check_state(state, self.N)
        if not isinstance(data, np.ndarray) or data.ndim != 1:
            raise ValueError("The moment data array is not one-dimensional")
        if data.shape[0] != self.n_obs:
            raise ValueError("The moment data array does not match the required size " + str(self.n_obs))
        if data.dtype != np.float64:
            raise ValueError("The moment data array does not match the required datatype: Float64")
        out = np.empty(self.n_obs)
        self._check(self._L.qcc_moments(self._c, np.ascontiguousarray(state).ctypes.data, out.ctypes.data))
        data[:] = out


class StepServer:
    """The step server of the reference's process model (qc_server_*): owns the GPU and one handle of
    `max_clients` envs; actor processes attach with load(..., server=name). run() serves on the calling
    thread; start() / stop() on a background thread."""

    def __init__(self, family: int | str = cfg.IHO, max_clients: int = 16, name: str | None = None, device: int = 0,
                 batch_wait_us: float = 40.0, **params):
        import os
        import torch

        from .core import make_params
        if isinstance(family, str):
            family = {v: k for k, v in cfg.FAMILY_NAMES.items()}[family]
        self.physics = cfg.DEFAULTS[family].with_(**params)
        self.name = name or f"/qcart_srv_{os.getpid()}"
        torch.cuda.init()
        self._L = _lib.lib()
        p = make_params(self.physics, max_clients, seed=0)
        h = ctypes.c_void_p()
        rc = self._L.qc_server_create(ctypes.byref(p), device, int(max_clients), self.name.encode(),
                                      float(batch_wait_us), ctypes.byref(h))
        if rc != 0:
            msg = (self._L.qc_last_error(None) or b"").decode()
            raise _lib.QCartError(rc, f"step server {self.name}: {msg}")
        self._h = h
        self._thread = None

    def run(self, seconds: float = 0.0):
        rc = self._L.qc_server_run(self._h, float(seconds))
        if rc != 0:
            raise _lib.QCartError(rc, (self._L.qc_server_last_error(self._h) or b"").decode())

    def start(self):
        import threading
        self._thread = threading.Thread(target=self.run, daemon=True)
        self._thread.start()
        return self

    def stop(self):
        if self._h:
            self._L.qc_server_stop(self._h)
        if self._thread is not None:
            self._thread.join()
            self._thread = None

    def stats(self):
        t, c = ctypes.c_int64(), ctypes.c_int64()
        self._L.qc_server_stats(self._h, ctypes.byref(t), ctypes.byref(c))
        tm = (ctypes.c_double * 4)()
        self._L.qc_server_timing(self._h, tm)
        rc, rl = ctypes.c_int64(), ctypes.c_int64()
        res = self._L.qc_server_resident(self._h, ctypes.byref(rc), ctypes.byref(rl))
        n = max(1, t.value)
        return {"ticks": t.value, "calls": c.value, "resident": bool(res == 1), "resident_calls": rc.value,
                "resident_launches": rl.value,
                "us_per_tick": {
            "batch_wait": tm[0] / n, "launch": tm[1] / n, "gpu": tm[2] / n, "publish": tm[3] / n}}

    def close(self):
        if getattr(self, "_h", None):
            self.stop()
            self._L.qc_server_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def load(family: int | str = cfg.IHO, device: int = 0, noise: str = "mt19937", server: str | None = None,
         **params) -> types.ModuleType:
    """Return a module-like object equivalent to the reference's compiled `simulation` extension.

    family: 0/'harmonic', 1/'inverted_harmonic', 2/'quartic', 3/'inverted_quartic'; params are the
    setupC.py macros (n_max, omega / x_max, grid_size, lambda_, mass, moment_order) and optionally
    gamma, time_steps, f_max, a_mode (defaults: the drivers' values, config.DEFAULTS). noise: 'mt19937'
    (the reference's stream, default) or 'philox'. server: the name of a running StepServer — the module's
    calls are then served by it (this process never touches the GPU; MT19937 noise)."""
    if isinstance(family, str):
        family = {v: k for k, v in cfg.FAMILY_NAMES.items()}[family]
    phys = cfg.DEFAULTS[family].with_(**params)
    key = (device, noise, server, tuple(sorted(phys.asdict().items())))
    if key not in _MODULES:
        if server is not None:
            if noise != "mt19937":
                raise ValueError("a step server draws the reference's MT19937 stream (noise='mt19937')")
            sim = _ServedSimulation(phys, server)
        else:
            sim = _Simulation(phys, device, noise)
        mod = types.ModuleType("simulation", "MI355X-native drop-in for the reference `simulation` module")
        for name in ("step", "simulate_10_steps", "set_seed", "check_settings", "x_expectation"):
            setattr(mod, name, getattr(sim, name))
        if not phys.fock:
            mod.get_moments = sim.get_moments
        else:
            # the Fock modules' method tables (IHO/simulation_i.cpp:618-631, HO/simulation.cpp:599-612), served too
            mod.Hamiltonian_dot_psi = sim.Hamiltonian_dot_psi
            mod.solve_ab = sim.solve_ab
        mod._impl = sim
        _MODULES[key] = mod
    return _MODULES[key]


def install(family: int | str = cfg.IHO, device: int = 0, noise: str = "mt19937", server: str | None = None,
            **params) -> types.ModuleType:
    """Register the drop-in as `simulation` in sys.modules, so the reference drivers'
    `__import__('simulation')` resolves to it (server: see load)."""
    mod = load(family, device, noise, server, **params)
    sys.modules["simulation"] = mod
    return mod


__all__ = ["load", "install", "StepServer", "pi"]
