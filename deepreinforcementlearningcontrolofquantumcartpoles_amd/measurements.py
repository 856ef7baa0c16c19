"""Measurement-record input mode: the per-env history of coarse-grained measurement
outcomes q that the reference's args.input == 'measurements' feeds to its network, kept on the device.

Reference: IHO/main_parallel.py:143-151 (sizes), :270-309 (the episode loop's lists);
HO/main_parallel.py:142-150, :259-292; the experience row layout read back by TrainDQN at
IHO/RL.py:175-192. The update is the HIP kernel behind qc_record (csrc/qcart_record.hip).
"""
from __future__ import annotations

from typing import Optional

import torch

from . import _lib as L
from . import config as cfg
from .core import Stepper, _ptr

DATA_PER_TIME_UNIT = 360 * 4          # num_of_data_per_time_unit (IHO/main_parallel.py:145)
N_PERIODS_TO_READ = {cfg.IHO: 2.0, cfg.HO: 1.5}   # IHO:144, HO:143


def default_read_length(family: int) -> int:
    """read_length = round(n_periods_to_read * 2 * num_of_data_per_time_unit) (IHO:148): 5760 / 4320."""
    return round(N_PERIODS_TO_READ[family] * 2 * DATA_PER_TIME_UNIT)


class MeasurementRecord:
    """hist [B][2][read_length] float32 (the network input: measurements newest first, and the force *
    input_scaling applied during each) and forces [B][K+1] (forces_to_store, newest first), updated in
    place once per control interval from the q outputs of Stepper.step(want_q=True)."""

    def __init__(self, stepper: Stepper, read_length: Optional[int] = None, coarse_grain: Optional[int] = None,
                 input_scaling: float = 1.0):
        ph = stepper.physics
        if ph.family not in N_PERIODS_TO_READ:
            raise ValueError("the 'measurements' input exists for the Fock drivers (harmonic, inverted harmonic)")
        if coarse_grain is None:
            if ph.time_steps % DATA_PER_TIME_UNIT:
                raise ValueError(f"time_steps {ph.time_steps} must be divisible by {DATA_PER_TIME_UNIT} (IHO:146)")
            coarse_grain = ph.time_steps // DATA_PER_TIME_UNIT
        self.st = stepper
        self.read_length = int(read_length or default_read_length(ph.family))
        self.coarse_grain = int(coarse_grain)
        self.interval = ph.control_interval
        self.input_scaling = float(input_scaling)
        self.row_len = L.check(L.lib().qc_record_row_len(self.read_length, self.interval, self.coarse_grain))
        self.m = self.interval // self.coarse_grain          # read_control_step_length (IHO:149)
        self.K = self.read_length // self.m
        B, dev = stepper.batch, stepper.device
        self.hist = torch.zeros((B, 2, self.read_length), dtype=torch.float32, device=dev)
        self.forces = torch.zeros((B, self.K + 1), dtype=torch.float32, device=dev)

    def record(self, q: torch.Tensor, actions: Optional[torch.Tensor] = None, default_action: Optional[int] = None,
               mode: Optional[torch.Tensor] = None, reward: Optional[torch.Tensor] = None,
               rows: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
        """Close one control interval: q [interval][B] fp64; mode [B] (0 skip, 1 record, 2 fresh history);
        rows [B][row_len] float32 receive the experience rows (reward column from reward [B] float32)."""
        st = self.st
        B = st.batch
        if q.dtype != torch.float64 or tuple(q.shape) != (self.interval, B) or not q.is_contiguous():
            raise ValueError(f"q must be a contiguous float64 ({self.interval}, {B}) tensor")
        if default_action is None:
            default_action = st.physics.n_actions // 2
        if actions is not None:
            actions = actions.to(device=st.device, dtype=torch.int32).contiguous()
            st._check_actions(actions)
        if mode is not None:
            mode = mode.to(device=st.device, dtype=torch.uint8).contiguous()
        if reward is not None:
            reward = reward.to(device=st.device, dtype=torch.float32).contiguous()
        if rows is not None and (rows.dtype != torch.float32 or tuple(rows.shape) != (B, self.row_len)
                                 or not rows.is_contiguous()):
            raise ValueError(f"rows must be a contiguous float32 ({B}, {self.row_len}) tensor")
        st._bind_stream()
        L.check(L.lib().qc_record(st._h, self.read_length, self.coarse_grain, self.input_scaling, _ptr(q),
                                  self.interval, _ptr(actions), int(default_action), _ptr(mode), _ptr(self.hist),
                                  _ptr(self.forces), _ptr(reward), _ptr(rows)), st._h)
        return rows


__all__ = ["MeasurementRecord", "default_read_length"]
