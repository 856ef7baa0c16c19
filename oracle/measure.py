"""Pure-Python restatement of the reference's measurement-record lists ('measurements' input).

TEST INFRASTRUCTURE ONLY: the checker of qc_record (csrc/qcart_record.hip), imported by tests/ only.
Follows IHO/main_parallel.py:270-309 (HO/main_parallel.py:259-292) list for list: measurements_cache,
measurements_input, forces_along_measurements_input, forces_to_store, and the experience row
np.hstack((measurements_input[::-1], forces_to_store[::-1], [last_action], [reward])) in float32.
Parity anchor: the reference's own list code (no outputs of it exist); small loops only.
"""
from __future__ import annotations

import numpy as np


class MeasureLists:
    def __init__(self, read_length: int, control_interval: int, coarse_grain: int, input_scaling: float):
        self.read_length = read_length
        self.cg = coarse_grain
        self.scale = input_scaling
        self.m = control_interval // coarse_grain            # read_control_step_length
        self.reset()

    def reset(self):
        """do_episode's initial lists (IHO:271-272)."""
        self.cache = []
        self.meas = list(np.zeros(self.read_length))
        self.frc_along = list(np.zeros(self.read_length))
        self.frc_store = list(np.zeros(self.read_length // self.m))

    def physics_step(self, q: float, force: float):
        """after simulation.step (IHO:284-288)."""
        self.cache.append(q)
        if len(self.cache) == self.cg:
            self.meas.append(sum(self.cache) / self.cg * self.scale)
            self.cache.clear()
            self.frc_along.append(force * self.scale)

    def control_step(self, force: float, last_action: int, reward: float):
        """the control step (IHO:263-283, :290-297): returns (experience row, network input)."""
        self.frc_store.append(force * self.scale)
        row = np.hstack((np.array(self.meas, dtype=np.float32)[::-1], np.array(self.frc_store, dtype=np.float32)[::-1],
                         np.array([last_action], dtype=np.float32), np.array([reward], dtype=np.float32)))
        self.meas, self.frc_along = self.meas[self.m:], self.frc_along[self.m:]
        self.frc_store = self.frc_store[1:]
        net_in = np.array([self.meas[::-1], self.frc_along[::-1]]).astype(np.float32)
        return row, net_in
