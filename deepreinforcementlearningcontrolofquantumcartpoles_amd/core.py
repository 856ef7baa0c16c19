"""Batched device stepper: a thin Python owner of one libqcart handle.

PyTorch is only plumbing here (device memory for psi / actions / observations and the HIP
stream); every physics operation runs in the HIP kernels behind include/qcart.h.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from . import _lib as L
from .config import Physics


def _ptr(t: Optional[torch.Tensor]):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def make_params(physics: Physics, batch: int, seed: int = 42, env_offset: int = 0,
                xth: float | None = None) -> L.QcParams:
    """qc_params of a handle for `physics` (the setupC.py macros + the drivers' step() arguments)."""
    p = L.QcParams()
    p.family = physics.family
    p.n_max = physics.n_max
    p.omega = physics.omega
    p.x_max = physics.x_max
    p.grid_size = physics.grid_size
    p.lambda_ = physics.lambda_
    p.mass = physics.mass
    p.moment_order = physics.moment_order
    p.a_mode = physics.a_mode
    p.precision = physics.precision
    p.gamma = physics.gamma
    p.dt = physics.dt
    p.f_max = physics.f_max
    p.n_actions = physics.n_actions
    p.batch = int(batch)
    p.env_offset = int(env_offset)
    p.seed = seed
    p.xth = physics.xth if (xth is None and physics.family == 3) else (xth or 0.0)
    return p


class Stepper:
    """B environments of one physical system on one device (one handle, one HIP stream)."""

    def __init__(self, physics: Physics, batch: int, device: int | str | torch.device = 0, seed: int = 42,
                 env_offset: int = 0, xth: float | None = None):
        if not torch.cuda.is_available():
            raise RuntimeError("libqcart needs a HIP device (no CPU fallback)")
        self.physics = physics
        self.batch = int(batch)
        self.device = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.env_offset = int(env_offset)
        p = make_params(physics, self.batch, seed, self.env_offset, xth)
        self._params = p
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            torch.cuda.init()
            L.check(L.lib().qc_create(ctypes.byref(p), self.device.index, ctypes.byref(h)))
        self._h = h
        self.N = L.lib().qc_dim(h)
        self.n_obs = L.lib().qc_n_obs(h)
        self.n_slots = physics.n_actions   # grows with add_force

    # ------------------------------------------------------------------ lifecycle
    def close(self):
        if getattr(self, "_h", None):
            L.lib().qc_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _bind_stream(self):
        s = torch.cuda.current_stream(self.device).cuda_stream
        L.check(L.lib().qc_set_stream(self._h, ctypes.c_void_p(s)), self._h)

    @property
    def state_dtype(self) -> torch.dtype:
        return torch.complex64 if self.physics.precision == 1 else torch.complex128

    def _check_psi(self, psi: torch.Tensor):
        if psi.dtype != self.state_dtype:
            name = "Complex64" if self.physics.precision == 1 else "Complex128"
            raise ValueError("The state array does not match the required datatype: " + name)
        if psi.dim() != 2 or psi.shape[1] != self.N or psi.shape[0] != self.batch:
            raise ValueError(f"The state array does not match the required size ({self.batch}, {self.N})")
        if psi.device != self.device or not psi.is_contiguous():
            raise ValueError("state must be a contiguous tensor on " + str(self.device))

    # ------------------------------------------------------------------ state helpers
    def new_state(self) -> torch.Tensor:
        return torch.zeros((self.batch, self.N), dtype=self.state_dtype, device=self.device)

    def set_seed(self, seed: int):
        """Philox noise keyed by seed, every env's counter back to 0 (qc_set_seed)."""
        L.check(L.lib().qc_set_seed(self._h, seed), self._h)

    def set_seed_mt19937(self, seeds):
        """The reference's noise stream (qc_set_seed_mt19937): env e draws from MT19937 seeded like
        vslNewStream(VSL_BRNG_MT19937, seeds[e]) with MKL's Box-Muller transform. seeds: an int (every
        env) or a sequence / tensor of B uint32 values."""
        if isinstance(seeds, int):
            seeds = [seeds] * self.batch
        t = torch.as_tensor(seeds, dtype=torch.int64)
        if t.shape != (self.batch,):
            raise ValueError(f"seeds must have shape ({self.batch},)")
        t = (t & 0xFFFFFFFF).to(torch.int64)
        # uint32 bit patterns in an int32 tensor (torch has no uint32 arithmetic on every backend)
        t = torch.where(t >= 2 ** 31, t - 2 ** 32, t).to(torch.int32).to(self.device).contiguous()
        self._bind_stream()
        L.check(L.lib().qc_set_seed_mt19937(self._h, _ptr(t)), self._h)
        torch.cuda.current_stream(self.device).synchronize()

    @property
    def noise_mode(self) -> str:
        return "mt19937" if L.lib().qc_noise_mode(self._h) == L.QC_NOISE_MT19937 else "philox"

    @property
    def step_counter(self) -> int:
        """env 0's Philox counter (every env keeps its own: env_counters)."""
        self._bind_stream()
        return int(L.lib().qc_get_step_counter(self._h))

    @step_counter.setter
    def step_counter(self, v: int):
        self._bind_stream()
        L.check(L.lib().qc_set_step_counter(self._h, int(v)), self._h)

    def env_counters(self, new: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Per-env Philox counters (int64 [B] copy); new replaces them (checkpoint / resume)."""
        out = torch.empty((self.batch,), dtype=torch.int64, device=self.device)
        if new is not None:
            new = new.to(device=self.device, dtype=torch.int64).contiguous()
            if new.shape != (self.batch,):
                raise ValueError(f"counters must have shape ({self.batch},)")
        self._bind_stream()
        L.check(L.lib().qc_env_counters(self._h, _ptr(out), _ptr(new)), self._h)
        return out

    def mt19937_state(self, new: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Per-env MT19937 states (int32 [B][qc_mt19937_words] copy of the uint32 words); new replaces them."""
        W = L.lib().qc_mt19937_words()
        out = torch.empty((self.batch, W), dtype=torch.int32, device=self.device)
        if new is not None:
            new = new.to(device=self.device, dtype=torch.int32).contiguous()
            if new.shape != (self.batch, W):
                raise ValueError(f"state must have shape ({self.batch}, {W})")
        self._bind_stream()
        L.check(L.lib().qc_mt19937_state(self._h, _ptr(out), _ptr(new)), self._h)
        return out

    def set_dynamics(self, dt: float, gamma: float):
        L.check(L.lib().qc_set_dynamics(self._h, dt, gamma), self._h)

    def add_force(self, force: float) -> int:
        slot = L.check(L.lib().qc_add_force(self._h, float(force)), self._h)
        self.n_slots = max(self.n_slots, slot + 1)
        return slot

    def group_layout(self):
        """(single-slot workgroups, two-slot workgroups) of the last grouped step() call: int32 numpy arrays
        [n][envs per workgroup] of env ids, -1 = idle wave (qc_group_layout; synchronises)."""
        import numpy as np
        g = int(L.lib().qc_step_group_size(self._h))
        order = np.full(((self.batch + g - 1) // g + 65) * g, -1, np.int32)
        mixed = np.full(64 * g, -1, np.int32)
        n_mixed = L.check(L.lib().qc_group_layout(self._h, order.ctypes.data, order.size, mixed.ctypes.data,
                                                  mixed.size), self._h)
        return order.reshape(-1, g), mixed[:n_mixed * g].reshape(-1, g)

    def scan_levels(self, action: int):
        f, b = ctypes.c_int32(), ctypes.c_int32()
        L.check(L.lib().qc_scan_levels(self._h, action, ctypes.byref(f), ctypes.byref(b)), self._h)
        return f.value, b.value

    # ------------------------------------------------------------------ hot path
    def step(self, psi: torch.Tensor, actions: Optional[torch.Tensor] = None, n_steps: int = 1,
             default_action: int | None = None, noise: Optional[torch.Tensor] = None,
             env_steps: Optional[torch.Tensor] = None, want_q: bool = False,
             want_fail: bool = True, want_term: bool = False, want_obs: bool = False) -> dict:
        """Advance every env n_steps physics steps in place (the reference's simulation.step,
        fused). Returns a dict of device tensors (q, x_mean, fail_step, term_step, obs)."""
        self._check_psi(psi)
        B = self.batch
        if actions is not None:
            self._check_actions(actions)
            actions = actions.contiguous()
        if default_action is None:
            default_action = self.physics.n_actions // 2
        if env_steps is not None:
            if env_steps.dtype != torch.int32 or env_steps.shape != (B,) or env_steps.device != self.device:
                raise ValueError("env_steps must be an int32 tensor of shape (B,) on the handle's device")
            env_steps = env_steps.contiguous()
        if noise is not None:
            if noise.dtype != torch.float64 or tuple(noise.shape) != (n_steps, B, 2) or noise.device != self.device:
                raise ValueError("noise must be float64 (n_steps, B, 2) on the handle's device")
            noise = noise.contiguous()
        out = {}
        dev = self.device
        q = torch.empty((n_steps, B), dtype=torch.float64, device=dev) if want_q else None
        xm = torch.empty((n_steps, B), dtype=torch.float64, device=dev) if want_q else None
        fs = torch.empty((B,), dtype=torch.int32, device=dev) if want_fail else None
        ts = torch.empty((B,), dtype=torch.int32, device=dev) if want_term else None
        ob = torch.empty((B, self.n_obs), dtype=torch.float64, device=dev) if want_obs else None
        self._bind_stream()
        L.check(L.lib().qc_step(self._h, _ptr(psi), _ptr(actions), int(default_action), int(n_steps),
                                _ptr(env_steps), _ptr(noise),
                                _ptr(q), _ptr(xm), _ptr(fs), _ptr(ts), _ptr(ob)), self._h)
        if want_q:
            out["q"], out["x_mean"] = q, xm
        if want_fail:
            out["fail_step"] = fs
        if want_term:
            out["term_step"] = ts
        if want_obs:
            out["obs"] = ob
        return out

    def _check_actions(self, actions: torch.Tensor):
        """int32 (B,) on the device. The values must be valid slots (the reference's convert_to_force has no
        other actions); that check runs on the device without a stream sync (qc_step's grouping kernel raises
        an error word) and is reported by check(), which every synchronising method calls."""
        if actions.dtype != torch.int32 or actions.shape != (self.batch,) or actions.device != self.device:
            raise ValueError("actions must be an int32 tensor of shape (B,) on the handle's device")

    def check(self):
        """Raise the deferred input errors of earlier step() calls (qc_take_errors; synchronises the stream)."""
        self._bind_stream()
        if L.lib().qc_take_errors(self._h) != 0:
            msg = L.lib().qc_last_error(self._h)
            raise ValueError(f"actions must lie in [0, {self.n_slots}): {msg.decode() if msg else ''}")

    def wavefunction_len(self) -> int:
        return L.check(L.lib().qc_wavefunction_len(self._h), self._h)

    def wavefunction_obs(self, psi: torch.Tensor, input_scaling: float = 1.0) -> torch.Tensor:
        """get_data_wavefunction(state) * input_scaling (float32 [B][wavefunction_len()]: HO state[:-10], IHO
        state[:-20], grid state[10:-10]; qc_wavefunction_obs)."""
        self._check_psi(psi)
        out = torch.empty((self.batch, self.wavefunction_len()), dtype=torch.float32, device=self.device)
        self._bind_stream()
        L.check(L.lib().qc_wavefunction_obs(self._h, _ptr(psi), float(input_scaling), _ptr(out)), self._h)
        return out

    def moments(self, psi: torch.Tensor) -> torch.Tensor:
        self._check_psi(psi)
        out = torch.empty((self.batch, self.n_obs), dtype=torch.float64, device=self.device)
        self._bind_stream()
        L.check(L.lib().qc_moments(self._h, _ptr(psi), _ptr(out)), self._h)
        return out

    def x_expectation(self, psi: torch.Tensor) -> torch.Tensor:
        self._check_psi(psi)
        out = torch.empty((self.batch,), dtype=torch.float64, device=self.device)
        self._bind_stream()
        L.check(L.lib().qc_x_expectation(self._h, _ptr(psi), _ptr(out)), self._h)
        return out

    def outside_prob(self, psi: torch.Tensor, xth: float) -> torch.Tensor:
        self._check_psi(psi)
        out = torch.empty((self.batch,), dtype=torch.float64, device=self.device)
        self._bind_stream()
        L.check(L.lib().qc_outside_prob(self._h, _ptr(psi), float(xth), _ptr(out)), self._h)
        return out

    def boundary_fail(self, psi: torch.Tensor) -> torch.Tensor:
        self._check_psi(psi)
        out = torch.empty((self.batch,), dtype=torch.int32, device=self.device)
        self._bind_stream()
        L.check(L.lib().qc_boundary_fail(self._h, _ptr(psi), _ptr(out)), self._h)
        return out

    def energy(self, psi: torch.Tensor) -> torch.Tensor:
        self._check_psi(psi)
        out = torch.empty((self.batch,), dtype=torch.float64, device=self.device)
        self._bind_stream()
        L.check(L.lib().qc_energy(self._h, _ptr(psi), _ptr(out)), self._h)
        return out

    def hamiltonian_dot_psi(self, psi: torch.Tensor) -> None:
        """psi <- H psi in place (the force-free Hamiltonian; the reference's Hamiltonian_dot_psi)."""
        self._check_psi(psi)
        self._bind_stream()
        L.check(L.lib().qc_hamiltonian_dot_psi(self._h, _ptr(psi)), self._h)

    def phonon_number(self, psi: torch.Tensor) -> torch.Tensor:
        self._check_psi(psi)
        out = torch.empty((self.batch,), dtype=torch.float64, device=self.device)
        self._bind_stream()
        L.check(L.lib().qc_phonon_number(self._h, _ptr(psi), _ptr(out)), self._h)
        return out

    def control(self, psi: torch.Tensor, strategy: str | int = "LQG", con_parameter: float = 0.0,
                control_time: float | None = None, input_scaling: float = 1.0):
        """Analytic baseline controller per env (qc_control): returns (actions int32 [B], force fp64 [B]).
        strategy: 'LQG' (Fock args.LQG; grid LinearQuadratic), 'damping', 'semiclassical' (grid).
        control_time defaults to 1 / n_con (IHO/main_parallel.py:195, QO/controllers.py:5)."""
        self._check_psi(psi)
        s = L.CONTROL_STRATEGIES[strategy] if isinstance(strategy, str) else int(strategy)
        if control_time is None:
            control_time = 1.0 / self.physics.n_con
        act = torch.empty((self.batch,), dtype=torch.int32, device=self.device)
        force = torch.empty((self.batch,), dtype=torch.float64, device=self.device)
        self._bind_stream()
        L.check(L.lib().qc_control(self._h, _ptr(psi), s, float(con_parameter), float(control_time),
                                   float(input_scaling), _ptr(act), _ptr(force)), self._h)
        return act, force

    def reset(self, psi: torch.Tensor, kind: int, mask: Optional[torch.Tensor] = None, arg0: float = 0.0,
              arg1: float = 0.0, arg2: float = 1.0, k: Optional[torch.Tensor] = None,
              mean: Optional[torch.Tensor] = None, std: Optional[torch.Tensor] = None):
        self._check_psi(psi)
        if mask is not None:
            mask = mask.to(device=self.device, dtype=torch.uint8).contiguous()
        for t in (k, mean, std):
            if t is not None and (t.dtype != torch.float64 or t.shape != (self.batch,)):
                raise ValueError("per-env reset parameters must be float64 (B,)")
        self._bind_stream()
        L.check(L.lib().qc_reset(self._h, _ptr(psi), kind, _ptr(mask), arg0, arg1, arg2, _ptr(k), _ptr(mean),
                                 _ptr(std)), self._h)

    def set_timing(self, on: bool = True):
        """HIP events around every k_step launch (qc_set_timing)."""
        L.check(L.lib().qc_set_timing(self._h, int(bool(on))), self._h)

    def step_kernel_time(self):
        """(summed k_step ms, launches) since the last read (synchronises the stream)."""
        ms, n = ctypes.c_double(), ctypes.c_int64()
        self._bind_stream()
        L.check(L.lib().qc_step_kernel_time(self._h, ctypes.byref(ms), ctypes.byref(n)), self._h)
        self.check()
        return ms.value, n.value

    def sync(self):
        L.check(L.lib().qc_sync(self._h), self._h)
        self.check()
