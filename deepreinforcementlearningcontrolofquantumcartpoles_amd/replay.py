"""Prioritized replay memory on the device: the reference's Memory / SumTree
(inverted harmonic oscillator/RL.py:234-475) with the same names and semantics, batched, resident in HBM.
The tree, the row storage and the policy scalars live on the GPU (csrc/qcart_replay.hip, C ABI
qc_replay_*); store / obtain_sample / batch_update launch kernels and never synchronise.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from . import _lib as L


def _ptr(t: Optional[torch.Tensor]):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


class PrioritizedReplay:
    """Memory(capacity, data_size, policy, passes_before_random) (RL.py:377-386) on `device`."""

    alpha = 0.2
    beta = 0.2
    beta_increment_per_sampling = 0.001
    abs_err_upper = 1.0

    def __init__(self, capacity: int, data_size: int, policy: str = "random", passes_before_random: float = 0.2,
                 device: int | str | torch.device = 0, seed: int = 0):
        if not torch.cuda.is_available():
            raise RuntimeError("libqcart needs a HIP device (no CPU fallback)")
        self.device = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        if policy not in ("sequential", "random"):
            raise ValueError("policy must be 'sequential' or 'random'")
        p = L.QcReplayParams()
        p.capacity = int(capacity)
        p.row_len = int(data_size)
        p.policy = 0 if policy == "sequential" else 1
        p.passes_before_random = float(passes_before_random)
        p.alpha = self.alpha
        p.beta = self.beta
        p.beta_increment = self.beta_increment_per_sampling
        p.abs_err_upper = self.abs_err_upper
        p.epsilon_scale = 1e-5
        p.seed = int(seed)
        self.capacity, self.data_size = int(capacity), int(data_size)
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            torch.cuda.init()
            L.check_replay(L.lib().qc_replay_create(ctypes.byref(p), self.device.index, ctypes.byref(h)))
        self._h = h
        self._len_ok = 0   # largest n for which len(memory) >= n has been seen

    def close(self):
        if getattr(self, "_h", None):
            L.lib().qc_replay_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _bind(self):
        s = torch.cuda.current_stream(self.device).cuda_stream
        L.check_replay(L.lib().qc_replay_set_stream(self._h, ctypes.c_void_p(s)), self._h)

    def _dev(self, t, dtype):
        return t.to(device=self.device, dtype=dtype).contiguous() if t is not None else None

    # ------------------------------------------------------------------ Memory API
    def store(self, rows: torch.Tensor, valid: Optional[torch.Tensor] = None):
        """Memory.store for every row (where valid): rows [n][data_size] float32."""
        rows = self._dev(rows, torch.float32)
        if rows.dim() != 2 or rows.shape[1] != self.data_size:
            raise ValueError(f"rows must be (n, {self.data_size})")
        valid = self._dev(valid, torch.uint8)
        self._bind()
        L.check_replay(L.lib().qc_replay_store(self._h, rows.shape[0], _ptr(valid), _ptr(rows)), self._h)

    def store_xp(self, last_obs: torch.Tensor, obs: torch.Tensor, action: torch.Tensor, reward: torch.Tensor,
                 valid: Optional[torch.Tensor] = None):
        """The 'xp' experience rows hstack((last_data, data, [last_action], [reward])) assembled in place."""
        last_obs, obs = self._dev(last_obs, torch.float32), self._dev(obs, torch.float32)
        action, reward = self._dev(action, torch.int32), self._dev(reward, torch.float32)
        valid = self._dev(valid, torch.uint8)
        n, d = obs.shape
        self._bind()
        L.check_replay(L.lib().qc_replay_store_xp(self._h, n, _ptr(valid), _ptr(last_obs), _ptr(obs), d,
                                                  _ptr(action), _ptr(reward)), self._h)

    def obtain_sample(self, n: int, u: Optional[torch.Tensor] = None, transitions: Optional[torch.Tensor] = None):
        """compiled_sampling: (tree_idx int32 [n], ISWeights float32 [n], transitions float32 [n][data_size]),
        or None while len(memory) < n (RL.py:424). u [n] fp64 injects the uniforms (np.random.rand).
        The length check synchronises only until it first passes (len never decreases)."""
        if n > self._len_ok:
            if len(self) < n:
                return None
            self._len_ok = n
        if transitions is None:
            transitions = torch.empty((n, self.data_size), dtype=torch.float32, device=self.device)
        idx = torch.empty((n,), dtype=torch.int32, device=self.device)
        w = torch.empty((n,), dtype=torch.float32, device=self.device)
        u = self._dev(u, torch.float64)
        self._bind()
        L.check_replay(L.lib().qc_replay_sample(self._h, int(n), _ptr(u), _ptr(transitions), _ptr(idx), _ptr(w)),
                       self._h)
        return idx, w, transitions

    def batch_update(self, tree_idx: torch.Tensor, abs_errors: torch.Tensor):
        tree_idx = self._dev(tree_idx, torch.int32)
        abs_errors = self._dev(abs_errors, torch.float32)
        self._bind()
        L.check_replay(L.lib().qc_replay_update(self._h, tree_idx.numel(), _ptr(tree_idx), _ptr(abs_errors)),
                       self._h)

    def clean(self):
        self._bind()
        L.check_replay(L.lib().qc_replay_rebuild(self._h), self._h)

    def stats(self) -> dict:
        s = L.QcReplayStats()
        L.check_replay(L.lib().qc_replay_stats(self._h, ctypes.byref(s)), self._h)
        return {k: getattr(s, k) for k, _ in L.QcReplayStats._fields_}

    def __len__(self) -> int:
        return int(self.stats()["len"])

    @property
    def total_p(self) -> float:
        return float(self.stats()["total_p"])

    def buffers(self):
        """(tree float64 [tree_size], data float32 [capacity][data_size]) as device tensors (views)."""
        st = self.stats()
        t, d = ctypes.c_void_p(), ctypes.c_void_p()
        L.check_replay(L.lib().qc_replay_buffers(self._h, ctypes.byref(t), ctypes.byref(d)), self._h)
        return _view(t.value, st["tree_size"], torch.float64, self.device), \
            _view(d.value, self.capacity * self.data_size, torch.float32, self.device).view(self.capacity, self.data_size)


def _view(addr: int, n: int, dtype, device) -> torch.Tensor:
    """A torch tensor viewing device memory owned by libqcart (__cuda_array_interface__; copy to keep)."""
    elt = torch.empty(0, dtype=dtype).element_size()

    class _A:
        __cuda_array_interface__ = {"shape": (n,), "typestr": {8: "<f8", 4: "<f4"}[elt], "data": (addr, False),
                                    "version": 3, "strides": None}
    return torch.as_tensor(_A(), device=device)
