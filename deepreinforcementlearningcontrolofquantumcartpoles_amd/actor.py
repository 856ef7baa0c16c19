"""Batched DQN actor on the device.

The reference evaluates its deep-Q network for the actors in one inference process that collects the
actors' inputs through pipes and answers with `action_values.max(1)[1]`
(inverted harmonic oscillator/main_parallel.py:414-440), while each actor applies its epsilon-greedy
choice (main_parallel.py:208-219). `DQNActor` does both for a whole `BatchedEnv` batch in one HIP launch
(csrc/qcart_actor.hip, `qc_actor_act`): direct_DQN's fc1 -> fc2 -> fc31 -> fc41 on f32-input MFMA,
argmax, epsilon-greedy. The parameters are the reference module's state_dict tensors (RL.py:80-111,
layers.py), so a trained `direct_DQN` drops in through `DQNActor(net.state_dict())`.

    actor = DQNActor(net.state_dict(), device=0, seed=seed)
    obs = env.reset()
    while True:
        actions = actor.act(obs, eps=DQNActor.eps_threshold(steps_done))
        obs, reward, done, info = env.step(actions)
"""
from __future__ import annotations

import ctypes
import math
from typing import Mapping, Optional

import torch

from . import _lib as L

LAYERS = ("fc1", "fc2", "fc31", "fc41")
HIDDEN = (512, 256, 256)


def _layer_tensors(params: Mapping[str, torch.Tensor], name: str, dev: torch.device):
    """(weight, bias, weight_norm, sigma_w, sigma_b) of one layer as contiguous fp32 device tensors:
    Linear_weight_normalize (weight, bias, weight_norm) or FactorizedNoisy (u_w, u_b, sigma_w, sigma_b)."""
    def t(key):
        v = params[f"{name}.{key}"]
        return v.detach().to(device=dev, dtype=torch.float32).contiguous()
    if f"{name}.u_w" in params:
        return t("u_w"), t("u_b"), None, t("sigma_w"), t("sigma_b")
    return t("weight"), t("bias"), t("weight_norm").reshape(1), None, None


class DQNActor:
    """Device-side action selection for B envs with a reference direct_DQN's parameters."""

    def __init__(self, params: Mapping[str, torch.Tensor], data_length: int = 5, n_actions: int = 21,
                 max_batch: int = 65536, device: int | str | torch.device = 0, seed: int = 0):
        self.device = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("DQNActor runs on a HIP device only (no CPU fallback)")
        self.data_length, self.n_actions, self.max_batch = int(data_length), int(n_actions), int(max_batch)
        p = L.QcDqnParams()
        p.data_length, p.n_actions, p.max_batch, p.seed = self.data_length, self.n_actions, self.max_batch, int(seed)
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            L.check_actor(L.lib().qc_actor_create(ctypes.byref(p), self.device.index or 0, ctypes.byref(h)), None)
        self._h = h
        self.noise_len = int(L.lib().qc_actor_noise_len(h))
        self.counter = 0
        self._keep = []
        self.load(params)

    def close(self):
        if getattr(self, "_h", None):
            L.lib().qc_actor_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _bind_stream(self):
        s = torch.cuda.current_stream(self.device).cuda_stream
        L.check_actor(L.lib().qc_actor_set_stream(self._h, ctypes.c_void_p(s)), self._h)

    def load(self, params: Mapping[str, torch.Tensor]):
        """(Re)load fc1, fc2, fc31, fc41 from a state_dict (the trainer's periodic push,
        main_parallel.py:400-405). Noisy / weight-normalised layers are recognised by their keys."""
        layers = (L.QcDqnLayer * 4)()
        keep = []
        for i, name in enumerate(LAYERS):
            w, b, g, sw, sb = _layer_tensors(params, name, self.device)
            out_f = HIDDEN[i] if i < 3 else self.n_actions
            in_f = self.data_length if i == 0 else HIDDEN[i - 1]
            if tuple(w.shape) != (out_f, in_f):
                raise ValueError(f"{name}: weight shape {tuple(w.shape)} != {(out_f, in_f)}")
            keep += [w, b, g, sw, sb]
            layers[i].weight, layers[i].bias = w.data_ptr(), b.data_ptr()
            layers[i].weight_norm = g.data_ptr() if g is not None else None
            layers[i].sigma_w = sw.data_ptr() if sw is not None else None
            layers[i].sigma_b = sb.data_ptr() if sb is not None else None
        with torch.cuda.device(self.device):
            self._bind_stream()
            L.check_actor(L.lib().qc_actor_load(self._h, layers), self._h)
        self._keep = keep   # the prep kernels read them on the current stream

    @staticmethod
    def eps_threshold(steps_done: float, start: float = 0.1, end: float = 0.003,
                      decay: float = 18 * 100 * 300) -> float:
        """The actor's epsilon schedule (IHO/main_parallel.py:186-189,208-210; decay = n_con*100*300)."""
        return (start - end) * math.exp(-1.0 * steps_done / decay) + end

    def act(self, obs: torch.Tensor, eps: float = 0.0, noisy: bool = True, counter: Optional[int] = None,
            noise: Optional[torch.Tensor] = None, env_offset: int = 0, want_q: bool = False,
            want_random: bool = False):
        """Actions [B] int32 for obs [B, data_length] (fp32, the network input). noise: optional injected
        NoisyNet noise [B, noise_len] (already f-transformed, layers.py:77-79); else drawn in-kernel
        with Philox (seed, env_offset + e, counter). Returns actions, or (actions, extras) when q / random
        flags are requested."""
        if obs.dim() != 2 or obs.shape[1] != self.data_length:
            raise ValueError(f"obs must be [B, {self.data_length}]")
        B = obs.shape[0]
        if B > self.max_batch:
            raise ValueError(f"B = {B} exceeds max_batch = {self.max_batch}")
        obs = obs.to(device=self.device, dtype=torch.float32).contiguous()
        if counter is None:
            counter = self.counter
            self.counter += 1
        nz = None
        if noise is not None:
            if tuple(noise.shape) != (B, self.noise_len):
                raise ValueError(f"noise must be [B, {self.noise_len}]")
            nz = noise.to(device=self.device, dtype=torch.float32).contiguous()
        actions = torch.empty(B, dtype=torch.int32, device=self.device)
        q = torch.empty((B, self.n_actions), dtype=torch.float32, device=self.device) if want_q else None
        rnd = torch.empty(B, dtype=torch.int32, device=self.device) if want_random else None
        vp = ctypes.c_void_p
        with torch.cuda.device(self.device):
            self._bind_stream()
            L.check_actor(L.lib().qc_actor_act(
                self._h, B, int(env_offset), vp(obs.data_ptr()), 1 if noisy else 0,
                vp(nz.data_ptr()) if nz is not None else None, float(eps), int(counter),
                vp(actions.data_ptr()), vp(q.data_ptr()) if q is not None else None,
                vp(rnd.data_ptr()) if rnd is not None else None), self._h)
        if want_q or want_random:
            return actions, {"q": q, "random": rnd}
        return actions


def random_direct_dqn(data_length: int = 5, n_actions: int = 21, noisy_layers: int = 2, seed: int = 0,
                      device: str | torch.device = "cpu") -> dict:
    """Random-initialised parameters of the reference direct_DQN (RL.py:80-111) as a state_dict, with
    the reference's initialisers: nn.Linear's default for Linear_weight_normalize (weight_norm = the
    initial ||W||_F, layers.py:97-100) and FactorizedNoisy's kaiming-uniform u_w, zero u_b and
    sigma = 0.5 / sqrt(in) (layers.py:22-29). Synthetic weights for tests and benchmarks."""
    g = torch.Generator().manual_seed(seed)

    def linear(name, i, o):
        bound = 1.0 / math.sqrt(i)
        w = (torch.rand((o, i), generator=g) * 2 - 1) * bound
        b = (torch.rand(o, generator=g) * 2 - 1) * bound
        return {f"{name}.weight": w, f"{name}.bias": b, f"{name}.weight_norm": w.norm()}

    def noisy(name, i, o):
        bound = math.sqrt(6.0 / i)   # kaiming_uniform_, fan_in, relu gain
        s = 0.5 / math.sqrt(i)
        return {f"{name}.u_w": (torch.rand((o, i), generator=g) * 2 - 1) * bound,
                f"{name}.sigma_w": torch.full((o, i), s), f"{name}.u_b": torch.zeros(o),
                f"{name}.sigma_b": torch.full((o,), s)}

    p = {}
    p.update(linear("fc1", data_length, 512))
    p.update(linear("fc2", 512, 256))
    p.update(noisy("fc31", 256, 256) if noisy_layers >= 2 else linear("fc31", 256, 256))
    p.update(linear("fc32", 256, 128))
    p.update(noisy("fc41", 256, n_actions) if noisy_layers >= 1 else linear("fc41", 256, n_actions))
    p.update(linear("fc42", 128, 1))
    return {k: v.to(device=device, dtype=torch.float32) for k, v in p.items()}


M_LAYERS = ("conv1", "conv2", "conv3", "fc1", "fc21", "fc31")
M_CONV = ((2, 32, 13, 5), (32, 64, 11, 4), (64, 64, 9, 4))   # (in, out, kernel, stride), RL.py:36-45


def conv_out(n: int, k: int, s: int) -> int:
    """calculate_next_layer_dim (IHO/RL.py:49-50)."""
    return (n - (k - 1) + (s - 1)) // s


def measurement_flat_len(read_length: int) -> int:
    n = read_length
    for _, _, k, s in M_CONV:
        n = conv_out(n, k, s)
    return 64 * n


class MeasurementActor:
    """Device-side action selection for B envs with a reference DQN_measurement's parameters (the
    'measurements' input, IHO/RL.py:29-78): obs = MeasurementRecord.hist [B, 2, read_length]."""

    def __init__(self, params: Mapping[str, torch.Tensor], read_length: int = 5760, n_actions: int = 21,
                 max_batch: int = 65536, device: int | str | torch.device = 0, seed: int = 0, chunk: int = 0):
        self.device = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("MeasurementActor runs on a HIP device only (no CPU fallback)")
        self.read_length, self.n_actions, self.max_batch = int(read_length), int(n_actions), int(max_batch)
        p = L.QcMdqnParams()
        p.read_length, p.n_actions, p.max_batch, p.seed, p.chunk = (self.read_length, self.n_actions,
                                                                     self.max_batch, int(seed), int(chunk))
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            L.check_mactor(L.lib().qc_mactor_create(ctypes.byref(p), self.device.index or 0, ctypes.byref(h)), None)
        self._h = h
        self.noise_len = int(L.lib().qc_mactor_noise_len(h))
        self.flat_len = int(L.lib().qc_mactor_flat_len(h))
        self.counter = 0
        self._keep = []
        self.load(params)

    def close(self):
        if getattr(self, "_h", None):
            L.lib().qc_mactor_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _bind_stream(self):
        s = torch.cuda.current_stream(self.device).cuda_stream
        L.check_mactor(L.lib().qc_mactor_set_stream(self._h, ctypes.c_void_p(s)), self._h)

    def load(self, params: Mapping[str, torch.Tensor]):
        layers = (L.QcDqnLayer * 6)()
        keep = []
        shapes = [(o, i * k) for i, o, k, _ in M_CONV] + [(256, self.flat_len), (256, 256), (self.n_actions, 256)]
        for j, name in enumerate(M_LAYERS):
            if j < 4:
                w = params[f"{name}.weight"].detach().to(device=self.device, dtype=torch.float32)
                w = w.reshape(w.shape[0], -1).contiguous()
                b = params[f"{name}.bias"].detach().to(device=self.device, dtype=torch.float32).contiguous()
                g = sw = sb = None
            else:
                w, b, g, sw, sb = _layer_tensors(params, name, self.device)
            if tuple(w.shape) != shapes[j]:
                raise ValueError(f"{name}: weight shape {tuple(w.shape)} != {shapes[j]}")
            keep += [w, b, g, sw, sb]
            layers[j].weight, layers[j].bias = w.data_ptr(), b.data_ptr()
            layers[j].weight_norm = g.data_ptr() if g is not None else None
            layers[j].sigma_w = sw.data_ptr() if sw is not None else None
            layers[j].sigma_b = sb.data_ptr() if sb is not None else None
        with torch.cuda.device(self.device):
            self._bind_stream()
            L.check_mactor(L.lib().qc_mactor_load(self._h, layers), self._h)
        self._keep = keep

    def act(self, obs: torch.Tensor, eps: float = 0.0, noisy: bool = True, counter: Optional[int] = None,
            noise: Optional[torch.Tensor] = None, env_offset: int = 0, want_q: bool = False,
            want_random: bool = False):
        """As DQNActor.act for obs [B, 2, read_length] (the measurement record)."""
        if obs.dim() != 3 or obs.shape[1] != 2 or obs.shape[2] != self.read_length:
            raise ValueError(f"obs must be [B, 2, {self.read_length}]")
        B = obs.shape[0]
        if B > self.max_batch:
            raise ValueError(f"B = {B} exceeds max_batch = {self.max_batch}")
        obs = obs.to(device=self.device, dtype=torch.float32).contiguous()
        if counter is None:
            counter = self.counter
            self.counter += 1
        nz = None
        if noise is not None:
            if tuple(noise.shape) != (B, self.noise_len):
                raise ValueError(f"noise must be [B, {self.noise_len}]")
            nz = noise.to(device=self.device, dtype=torch.float32).contiguous()
        actions = torch.empty(B, dtype=torch.int32, device=self.device)
        q = torch.empty((B, self.n_actions), dtype=torch.float32, device=self.device) if want_q else None
        rnd = torch.empty(B, dtype=torch.int32, device=self.device) if want_random else None
        vp = ctypes.c_void_p
        with torch.cuda.device(self.device):
            self._bind_stream()
            L.check_mactor(L.lib().qc_mactor_act(
                self._h, B, int(env_offset), vp(obs.data_ptr()), 1 if noisy else 0,
                vp(nz.data_ptr()) if nz is not None else None, float(eps), int(counter),
                vp(actions.data_ptr()), vp(q.data_ptr()) if q is not None else None,
                vp(rnd.data_ptr()) if rnd is not None else None), self._h)
        if want_q or want_random:
            return actions, {"q": q, "random": rnd}
        return actions


def random_dqn_measurement(read_length: int = 5760, n_actions: int = 21, seed: int = 0,
                           device: str | torch.device = "cpu") -> dict:
    """Random-initialised parameters of the reference DQN_measurement (RL.py:29-78) as a state_dict:
    PyTorch's default Conv1d / Linear initialisers (conv biases zeroed, RL.py:46-48), FactorizedNoisy as
    in random_direct_dqn, and the unused mean branch fc22 / fc32. Synthetic weights for tests / benches."""
    g = torch.Generator().manual_seed(seed)

    def uni(shape, bound):
        return (torch.rand(shape, generator=g) * 2 - 1) * bound

    p = {}
    for j, (ci, co, k, _) in enumerate(M_CONV):
        bound = 1.0 / math.sqrt(ci * k)
        p[f"conv{j + 1}.weight"] = uni((co, ci, k), bound)
        p[f"conv{j + 1}.bias"] = torch.zeros(co)
    flat = measurement_flat_len(read_length)
    p["fc1.weight"] = uni((256, flat), 1.0 / math.sqrt(flat))
    p["fc1.bias"] = uni((256,), 1.0 / math.sqrt(flat))

    def noisy(name, i, o):
        s = 0.5 / math.sqrt(i)
        return {f"{name}.u_w": uni((o, i), math.sqrt(6.0 / i)), f"{name}.sigma_w": torch.full((o, i), s),
                f"{name}.u_b": torch.zeros(o), f"{name}.sigma_b": torch.full((o,), s)}

    def linear(name, i, o):
        w = uni((o, i), 1.0 / math.sqrt(i))
        return {f"{name}.weight": w, f"{name}.bias": uni((o,), 1.0 / math.sqrt(i)), f"{name}.weight_norm": w.norm()}

    p.update(noisy("fc21", 256, 256))
    p.update(noisy("fc31", 256, n_actions))
    p.update(linear("fc22", 256, 128))
    p.update(linear("fc32", 128, 1))
    return {k: v.to(device=device, dtype=torch.float32) for k, v in p.items()}
