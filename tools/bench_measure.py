#!/usr/bin/env python3
"""Measurement-record input mode on one GPU (SURVEY §8f rank 3 measured in place): BatchedEnv IHO N = 512,
input='measurements' (read_length 5760), actions from the device LQG controller (qc_control), K control
steps with auto-reset. Times the loop and, with HIP events on the env's stream, one qc_record call alone
(the record kernel: 2 x 5760 float32 history shifted in place + the 5915-float experience row per env).
Prints one JSON line. usage: python tools/bench_measure.py [--batch B] [--steps K]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from deepreinforcementlearningcontrolofquantumcartpoles_amd import config as cfg  # noqa: E402
from deepreinforcementlearningcontrolofquantumcartpoles_amd.env import BatchedEnv  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=1)
    args = ap.parse_args()
    B = args.batch
    ph = cfg.DEFAULTS[cfg.IHO].with_(n_max=511)
    env = BatchedEnv(ph, B, 0, seed=1, input="measurements")
    env.reset()
    for it in range(args.warmup + args.steps):
        if it == args.warmup:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        env.step(env.analytic_actions("LQG"))
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    K = args.steps
    # the record kernel alone: one more interval's q stream, recorded R times into the live buffers
    rec = env.rec
    q = torch.randn((ph.control_interval, B), dtype=torch.float64, device=env.dev)
    reward = torch.ones(B, dtype=torch.float32, device=env.dev)
    a = torch.full((B,), 10, dtype=torch.int32, device=env.dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    R = 10
    rec.record(q, a, reward=reward, rows=env.rows)
    e0.record()
    for _ in range(R):
        rec.record(q, a, reward=reward, rows=env.rows)
    e1.record()
    e1.synchronize()
    rec_ms = e0.elapsed_time(e1) / R
    bytes_per_env = 4 * (2 * 2 * rec.read_length + rec.row_len + 2 * (rec.K + 1)) + 8 * ph.control_interval
    print(json.dumps({"metric": "measurement-mode loop RL steps/s (BatchedEnv IHO N=512, input='measurements', LQG)",
                      "value": B * K / dt, "unit": "decisions/s", "env_steps_per_s": B * K * ph.control_interval / dt,
                      "batch": B, "control_steps": K, "ms_per_control_step": dt / K * 1e3,
                      "record_ms": rec_ms, "record_share": rec_ms * K / (dt * 1e3),
                      "record_GBps": bytes_per_env * B / (rec_ms * 1e-3) / 1e9,
                      "record_bytes_per_env": bytes_per_env,
                      "data": "synthetic: |0> resets, LQG actions"}), flush=True)


if __name__ == "__main__":
    main()
