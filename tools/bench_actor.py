#!/usr/bin/env python3
"""Measurement of the device DQN actor: one qc_actor_act over the per-GPU metric batch
(65 536 envs, 'xp' input, noisy_layers = 2, in-kernel NoisyNet noise), timed with HIP events on the
actor's stream; roofline against the f32-input MFMA peak (MI355X_MICROARCH.md: 157.3 TF).
Prints one JSON line. usage: python tools/bench_actor.py [--batch B] [--reps K]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from deepreinforcementlearningcontrolofquantumcartpoles_amd.actor import DQNActor, random_direct_dqn  # noqa: E402

PEAK_F32_MFMA = 157.3e12


def flops_per_env(data_length=5, n_actions=21, noisy=True):
    macs = data_length * 512 + 512 * 256 + (2 if noisy else 1) * 256 * 256 + (2 if noisy else 1) * 256 * n_actions
    return 2 * macs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    B = args.batch
    actor = DQNActor({k: v.cuda() for k, v in random_direct_dqn(seed=1).items()}, max_batch=B, seed=2)
    obs = torch.randn((B, 5), device="cuda")
    actor.act(obs, eps=0.01)
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(args.reps):
        actor.act(obs, eps=0.01)
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.reps
    fl = flops_per_env() * B
    print(json.dumps({"metric": "DQN actor decisions/s (one qc_actor_act over the batch)", "value": B / ms * 1e3,
                      "unit": "decisions/s", "batch": B, "ms_per_call": ms, "dtype": "f32",
                      "roofline": {"bound": "mfma", "achieved": fl / (ms * 1e-3) / 1e12,
                                   "peak": PEAK_F32_MFMA / 1e12, "unit": "TFLOP/s",
                                   "frac": fl / (ms * 1e-3) / PEAK_F32_MFMA, "flops_per_decision": flops_per_env()},
                      "note": "time includes the in-kernel NoisyNet noise draw (k_actor_noise) and epsilon-greedy"}),
          flush=True)


if __name__ == "__main__":
    main()
