"""BatchedEnv: the reference actors' episode loop (Control.do_episode) for B environments at once,
on device tensors, one control interval per step().

Reference semantics reproduced per family ('xp' observation input):
  * cartpoles (IHO, IQO): IHO/main_parallel.py:227-268, IQO/main_parallel.py:172-222
      - reset: IHO |0>, IQO Gaussian_packet(inf, 0, 1); force 0 for the first control interval
        (no control at the zero-th step), first decision at i = control_interval
      - done when the boundary Fail flag fired during the interval (numerical_failure) or, at the
        control step, |<x>| > xth = F_max (IHO) / the outside probability exceeded 0.5 at any
        physics step (IQO, checked every step); reward row value 1 (alive) or failing_reward (-1)
  * cooling (HO, QO): HO/main_parallel.py:222-292, QO/main_parallel.py:169-232
      - reset: HO |0>; QO Gaussian(k ~ U[-0.3,0.3]) evolved U[15,20] time units at F = 0, redrawn
        until energy < 7.5 and no Fail (QO/main_parallel.py:177-198)
      - first decision at i = control_interval after a zero-force interval (HO:238, like the
        cartpoles) / at i = 0 (QO:208); at each control step the transition is stored with reward
        -phonon*scale (HO) / -energy*scale (QO) while phonon <= cutoff / energy < cutoff and no Fail;
        otherwise the episode ends without storing it; the episode is truncated at t_max = 100
The experience row layout is the reference's: [last_obs, obs, last_action, reward]
(IHO/main_parallel.py:250-257), so the deep-Q consumer drops in unchanged. With input='wavefunction'
the observation is get_data_wavefunction(state) * input_scaling: float32 hstack(Re, Im) of state[:-10]
(HO, HO/main_parallel.py:132-134), state[:-20] (IHO, IHO/main_parallel.py:133-135) or state[10:-10]
(grid, IQO/main_parallel.py:136-137)
(qc_wavefunction_obs). With input='measurements'
(HO, IHO; IHO/main_parallel.py:143-151,270-309) the observation is the device measurement record
[B][2][read_length] (measurements.MeasurementRecord, updated in place by the qc_record kernel) and the
experience rows [B][row_len] come from the same kernel (info['rows']).

Auto-reset modes (cartpoles, 'xp' input):
  * reset="immediate" (default): a finished env is reset and runs its zero-force first interval inside the same
    step() call, so the returned obs of a done env is already the next episode's first observation (the terminal
    one is info['terminal_obs']) — the reference actor's own interleaving; one more (partial) step launch and a few
    host synchronisations per call.
  * reset="deferred": a finished env returns its terminal obs and runs its reset interval (|0> / the IQO packet at
    F = 0) in the NEXT call, inside the same step launch as the other envs (its action of that call is ignored,
    info['reset'] marks it, no valid transition); the per-control-step bookkeeping (reward, done, return, episode
    time, the finished-episode ring) is one device kernel (qc_env_tail) and the call never synchronises with the
    host. Every env's own sequence — reset, zero-force interval, decisions on its observations, per-env noise — is
    the immediate mode's (tests/test_gpu_env.py: per-env episodes bitwise equal); only the calls they fall in
    differ, and every call advances every env exactly one control interval.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from . import config as cfg
from .core import Stepper
from .measurements import MeasurementRecord


class BatchedEnv:
    def __init__(self, physics: cfg.Physics, batch: int, device: int | str | torch.device = 0, seed: int = 0,
                 env_offset: int = 0, input_scaling: float = 1.0, failing_reward: float = -1.0,
                 reward_multiply: float = 1.0, t_max: float = 100.0, phonon_cutoff: float = 20.0,
                 energy_cutoff: float = 12.0, init_energy_cutoff: float = 7.5, auto_reset: bool = True,
                 reset_kind: str = "reference", input: str = "xp", read_length: Optional[int] = None,
                 reset: str = "immediate"):
        self.ph = physics
        self.B = int(batch)
        self.st = Stepper(physics, self.B, device, seed=seed, env_offset=env_offset)
        self.dev = self.st.device
        self.psi = self.st.new_state()
        self.ci = physics.control_interval
        self.half = physics.n_actions // 2
        self.input_scaling = input_scaling
        self.failing_reward = failing_reward
        self.reward_multiply = reward_multiply
        self.t_max = t_max
        self.phonon_cutoff = phonon_cutoff
        self.energy_cutoff = energy_cutoff
        self.init_energy_cutoff = init_energy_cutoff
        self.auto_reset = auto_reset
        self.reset_kind = reset_kind
        self.cartpole = physics.family in (cfg.IHO, cfg.IQO)
        # no control at the zero-th step: the first decision follows one zero-force interval (IHO:250,
        # IQO:201, HO:238); QO decides at i = 0 (QO:208)
        self.first_interval = physics.family != cfg.QO
        if input not in ("xp", "wavefunction", "measurements"):
            raise ValueError("input must be 'xp', 'wavefunction' or 'measurements'")
        if input == "measurements" and not physics.fock:
            raise ValueError("the 'measurements' input exists for the Fock families (HO, IHO) only")
        self.input = input
        if reset not in ("immediate", "deferred"):
            raise ValueError("reset must be 'immediate' or 'deferred'")
        if reset == "deferred" and not (self.cartpole and input == "xp" and auto_reset):
            raise ValueError("reset='deferred' is built for the cartpoles (IHO, IQO) with the 'xp' input and auto_reset")
        self.reset_mode = reset
        self._pending = torch.zeros(self.B, dtype=torch.uint8, device=self.dev)
        self._calls = 0
        self.rec = None
        if input == "measurements":
            self.rec = MeasurementRecord(self.st, read_length, input_scaling=input_scaling)
            self.rows = torch.empty((self.B, self.rec.row_len), dtype=torch.float32, device=self.dev)
        self.gen = torch.Generator(device=self.dev).manual_seed(int(seed) * 7919 + int(env_offset))
        z = lambda dt: torch.zeros(self.B, dtype=dt, device=self.dev)  # noqa: E731
        self.t = z(torch.float64)                 # episode time
        self.steps = z(torch.int64)               # physics steps in the episode
        self.last_action = torch.full((self.B,), self.half, dtype=torch.int32, device=self.dev)
        obs_len = self.st.wavefunction_len() if input == "wavefunction" else self.st.n_obs
        self.obs = (self.rec.hist if self.rec is not None else
                    torch.zeros((self.B, obs_len), dtype=torch.float32, device=self.dev))
        self.episode_return = z(torch.float64)
        # finished episodes (return, length) compacted on the device into a ring of _fin_cap entries
        # (slot _fin_cap is the sink of the not-finished envs): no boolean indexing, no dynamic shapes and
        # no host copy per step; read through finished_returns
        self._fin_cap = max(1 << 16, 16 * self.B)
        self._fin = torch.zeros((2, self._fin_cap + 1), dtype=torch.float64, device=self.dev)
        self._fin_n = torch.zeros((), dtype=torch.int64, device=self.dev)
        self._fin_read = 0
        self._fin_host: list = []

    @property
    def finished_returns(self) -> list:
        """(returns, lengths) float64 CPU tensors of the episodes finished so far, one entry per read
        that found new ones (the reference's per-actor result queue, main_parallel.py:300-327). At most
        the last _fin_cap episodes between two reads are kept."""
        n = int(self._fin_n)
        if n > self._fin_read:
            lo = max(self._fin_read, n - self._fin_cap)
            idx = torch.arange(lo, n, device=self.dev) % self._fin_cap
            vals = self._fin[:, idx].cpu()
            self._fin_host.append((vals[0], vals[1]))
            self._fin_read = n
        return self._fin_host

    def _push_finished(self, done: torch.Tensor, ret: torch.Tensor, length: torch.Tensor):
        """Append the finished episodes (env order) to the device ring, no host sync."""
        pos = self._fin_n + torch.cumsum(done, 0) - 1
        slot = torch.where(done, pos % self._fin_cap, torch.full_like(pos, self._fin_cap))
        self._fin[0].index_copy_(0, slot, ret)   # duplicates only into the sink
        self._fin[1].index_copy_(0, slot, length)
        self._fin_n += done.sum()

    # ------------------------------------------------------------------ observation
    def _observe(self) -> torch.Tensor:
        if self.input == "wavefunction":
            return self.st.wavefunction_obs(self.psi, self.input_scaling)
        return self.st.moments(self.psi).to(torch.float32) * self.input_scaling

    def _quantity(self) -> torch.Tensor:
        """cooling reward quantity: phonon number (HO) / energy (QO)."""
        if self.ph.family == cfg.HO:
            return self.st.phonon_number(self.psi)
        return self.st.energy(self.psi)

    # ------------------------------------------------------------------ reset
    def _reset_states(self, mask: torch.Tensor):
        m8 = mask.to(torch.uint8)
        fam = self.ph.family
        if fam in (cfg.HO, cfg.IHO):
            if self.reset_kind == "synthetic":
                self.st.reset(self.psi, 1, mask=m8, arg0=16)
            else:
                self.st.reset(self.psi, 0, mask=m8)
        elif fam == cfg.IQO:
            self.st.reset(self.psi, 2, mask=m8, arg0=0.0, arg1=0.0, arg2=1.0)
        else:
            self._reset_quartic_cooling(mask)

    def _reset_quartic_cooling(self, mask: torch.Tensor):
        """QO/main_parallel.py:177-198: random-k packet, free evolution for U[15,20] time units, redrawn
        until energy < init_energy_cutoff and no Fail."""
        todo = mask.clone()
        dt = self.ph.dt
        rounds = 0
        while bool(todo.any()):
            rounds += 1
            if rounds > 1000:   # the reference redraws without bound; a broken scheme would spin forever
                raise RuntimeError("quartic cooling reset: no acceptable initial state after 1000 redraws")
            k = (torch.rand(self.B, generator=self.gen, device=self.dev, dtype=torch.float64) * 0.6 - 0.3)
            mu = torch.zeros(self.B, dtype=torch.float64, device=self.dev)
            sg = torch.ones(self.B, dtype=torch.float64, device=self.dev)
            self.st.reset(self.psi, 2, mask=todo.to(torch.uint8), k=k, mean=mu, std=sg)
            init_t = torch.rand(self.B, generator=self.gen, device=self.dev, dtype=torch.float64) * 5.0 + 15.0
            budget = torch.where(todo, torch.ceil(init_t / dt).to(torch.int32), torch.zeros_like(init_t, dtype=torch.int32))
            failed = torch.zeros(self.B, dtype=torch.bool, device=self.dev)
            chunk = 1440
            while bool((budget > 0).any()):
                out = self.st.step(self.psi, None, chunk, default_action=self.half,
                                   env_steps=torch.clamp(budget, max=chunk).to(torch.int32))
                failed |= out["fail_step"] > 0
                budget = torch.clamp(budget - chunk, min=0)
            ok = (self._quantity() < self.init_energy_cutoff) & ~failed
            todo = todo & ~ok

    def reset(self, mask: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Start new episodes (all, or where mask); returns the observation at the first decision."""
        if mask is None:
            mask = torch.ones(self.B, dtype=torch.bool, device=self.dev)
        mask = mask.to(device=self.dev, dtype=torch.bool)
        self._pending.masked_fill_(mask, 0)   # (reset='deferred': a pending reset is done here instead)
        self._reset_states(mask)
        self.t = torch.where(mask, torch.zeros_like(self.t), self.t)
        self.steps = torch.where(mask, torch.zeros_like(self.steps), self.steps)
        self.episode_return = torch.where(mask, torch.zeros_like(self.episode_return), self.episode_return)
        self.last_action = torch.where(mask, torch.full_like(self.last_action, self.half), self.last_action)
        if self.first_interval:
            # no control at the zero-th step: one zero-force interval first (IHO:242-268, IQO:190-221,
            # HO:237-257). An episode that already ends at i = control_interval stores no transition
            # (i != control_interval guard, IHO:250) but is still reported with its length t (the
            # (experience, t, numerical_failure) / (t,) queue puts, IHO:312-313) and restarted here.
            fam = self.ph.family
            todo = mask.clone()
            while bool(todo.any()):
                budget = torch.where(todo, torch.full_like(self.last_action, self.ci), torch.zeros_like(self.last_action))
                out = self.st.step(self.psi, None, self.ci, default_action=self.half, env_steps=budget,
                                   want_term=(fam == cfg.IQO), want_obs=True, want_q=self.rec is not None)
                if self.rec is not None:   # the record starts at i = 0 from empty lists (IHO:271-272)
                    self.rec.record(out["q"], None, self.half, mode=todo.to(torch.uint8) * 2)
                bad = out["fail_step"] > 0
                if fam == cfg.IQO:
                    bad |= out["term_step"] >= 0
                elif fam == cfg.IHO:
                    bad |= out["obs"][:, 0].abs() > self.ph.xth
                else:   # HO: phonon > cutoff at the first control step ends the episode (HO:240-246)
                    bad |= self.st.phonon_number(self.psi) > self.phonon_cutoff
                bad &= todo
                if bool(bad.any()):
                    length = torch.where(mask, self.t + self.ci * self.ph.dt, self.t)
                    self._push_finished(bad, torch.zeros_like(self.t), length)
                    self._reset_states(bad)
                todo = bad
            self.t = torch.where(mask, self.t + self.ci * self.ph.dt, self.t)
            self.steps = torch.where(mask, self.steps + self.ci, self.steps)
        if self.rec is not None:
            self.obs = self.rec.hist
            return self.obs
        obs = self._observe()
        self.obs = torch.where(mask[:, None], obs, self.obs)
        return self.obs

    # ------------------------------------------------------------------ step
    def _step_deferred(self, actions: torch.Tensor):
        """reset='deferred': the envs finished in the previous call take their reset interval now (reset kernel +
        the zero force in the same step launch), then qc_env_tail does the bookkeeping on the device."""
        from . import _lib as L
        fam = self.ph.family
        pend = self._pending
        reset_now = pend.clone().view(torch.bool)
        self._reset_states(reset_now)   # the immediate mode's reset (reset_kind included), masked
        acts = torch.where(reset_now, torch.full_like(actions, self.half), actions)
        out = self.st.step(self.psi, acts, self.ci, want_fail=True, want_obs=True, want_term=(fam == cfg.IQO))
        B, n = self.B, self.st.n_obs
        obs = torch.empty((B, n), dtype=torch.float32, device=self.dev)
        reward = torch.empty(B, dtype=torch.float32, device=self.dev)
        done = torch.empty(B, dtype=torch.uint8, device=self.dev)
        valid = torch.empty(B, dtype=torch.uint8, device=self.dev)
        p = lambda t: t.data_ptr() if t is not None else None   # noqa: E731
        a = L.QcEnvTailArgs(B=B, kind=fam, n_obs=n, interval=self.ci, dt=self.ph.dt, xth=self.ph.xth,
                            input_scaling=self.input_scaling, failing_reward=self.failing_reward,
                            fail_step=p(out["fail_step"]), term_step=p(out.get("term_step")), obs=p(out["obs"]),
                            pending=p(pend), t=p(self.t), steps=p(self.steps), episode_return=p(self.episode_return),
                            obs32=p(obs), reward=p(reward), done=p(done), valid=p(valid), fin=p(self._fin),
                            fin_cap=self._fin_cap, fin_n=p(self._fin_n))
        self.st._bind_stream()
        L.check(L.lib().qc_env_tail(self.st._h, ctypes.byref(a)), self.st._h)
        last_obs = self.obs
        self.obs = obs
        self.last_action = acts
        self._calls += 1
        if self._calls % 16 == 0:   # deferred action-range errors, at most 16 calls late (synchronises)
            self.st.check()
        done_b = done.view(torch.bool)
        info = {"valid": valid.view(torch.bool), "reset": reset_now, "t": self.t.clone(), "last_obs": last_obs,
                "fail_step": out["fail_step"], "numerical_failure": done_b & (out["fail_step"] > 0)}
        return obs, reward, done_b, info

    def step(self, actions: torch.Tensor):
        """Apply per-env actions for one control interval. Returns (obs, reward, done, info):
        reward is the reference's stored reward-row value, info['valid'] marks transitions the
        reference would store, info['numerical_failure'] the Fail-terminated episodes."""
        actions = actions.to(device=self.dev, dtype=torch.int32).contiguous()
        if self.reset_mode == "deferred":
            return self._step_deferred(actions)
        last_obs = self.obs
        fam = self.ph.family
        out = self.st.step(self.psi, actions, self.ci, want_fail=True, want_obs=True,
                           want_term=(fam == cfg.IQO), want_q=self.rec is not None)
        fail = out["fail_step"] > 0
        if self.input == "wavefunction":
            obs = self.st.wavefunction_obs(self.psi, self.input_scaling)
        else:
            obs = out["obs"].to(torch.float32) * self.input_scaling
        self.t = self.t + self.ci * self.ph.dt
        self.steps = self.steps + self.ci
        if self.cartpole:
            numerical = fail                                     # Fail during the interval (IHO:243-267)
            if fam == cfg.IHO:
                out_of_bounds = out["obs"][:, 0].abs() > self.ph.xth   # |x_expectation| > xth (IHO:246)
            else:
                out_of_bounds = out["term_step"] >= 0                 # outside prob > 0.5 (IQO:199-200)
            done = numerical | out_of_bounds
            reward = torch.where(done, torch.full_like(self.t, self.failing_reward), torch.ones_like(self.t))
            valid = torch.ones_like(done)
        else:
            q = self._quantity()
            cutoff = self.phonon_cutoff if fam == cfg.HO else self.energy_cutoff
            ok = (q <= cutoff) if fam == cfg.HO else (q < cutoff)
            truncated = self.t >= self.t_max - 0.01 * self.ph.dt
            done = fail | ~ok | truncated
            reward = -q * self.reward_multiply
            valid = ~done
            numerical = fail
        self.episode_return = self.episode_return + torch.where(valid, reward, torch.zeros_like(reward))
        info = {"valid": valid, "numerical_failure": numerical & done, "t": self.t.clone(),
                "last_obs": last_obs if self.rec is None else None, "fail_step": out["fail_step"]}
        if self.rec is not None:
            # the continuous record of the two control steps, forces and (action, reward) (IHO:270-283)
            self.rec.record(out["q"], actions, self.half, reward=reward.to(torch.float32), rows=self.rows)
            info["rows"] = self.rows
            obs = self.rec.hist
        self.last_action = actions
        self.obs = obs
        self.st.check()   # deferred action-range errors of this interval's step (synchronises, as done.any() does)
        if bool(done.any()):
            if self.rec is None:   # measurement mode: the rows hold the terminal record
                info["terminal_obs"] = obs.clone()
            info["episode_return"] = self.episode_return.clone()
            info["episode_length"] = self.t.clone()
            self._push_finished(done, self.episode_return, self.t)
            if self.auto_reset:
                self.reset(done)
        return self.obs, reward.to(torch.float32), done, info

    def analytic_actions(self, strategy: str = "LQG", con_parameter: float = 0.0) -> torch.Tensor:
        """Actions of the reference's analytic baseline controllers for the current states (qc_control):
        Fock args.LQG on the 'xp' network input (IHO/main_parallel.py:194-206), grid
        args.control_strategy in {'LQG', 'damping', 'semiclassical'} (QO/main_parallel.py:165-181)."""
        # the 'xp' input hands the scaled network input to call_force; other inputs pass the unscaled
        # get_data_xp(state) (IHO:259-262)
        sc = self.input_scaling if self.input == "xp" else 1.0
        act, _ = self.st.control(self.psi, strategy, con_parameter, input_scaling=sc)
        return act

    @staticmethod
    def experience(last_obs: torch.Tensor, obs: torch.Tensor, action: torch.Tensor, reward: torch.Tensor):
        """Experience rows in the reference layout np.hstack((last_data, data, [last_action], [reward]))."""
        return torch.cat([last_obs, obs, action.to(torch.float32)[:, None], reward.to(torch.float32)[:, None]], 1)
