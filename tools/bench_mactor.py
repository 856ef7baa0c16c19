#!/usr/bin/env python3
"""Measurement of the measurement-input actor (DQN_measurement, qc_mactor_act) over the per-GPU batch
(65 536 envs, read_length 5760, in-kernel NoisyNet noise), timed with HIP events on its stream; roofline
against the f32-input MFMA peak (MI355X_MICROARCH.md: 157.3 TF). Prints one JSON line.
usage: python tools/bench_mactor.py [--batch B] [--reps K] [--chunk C]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from deepreinforcementlearningcontrolofquantumcartpoles_amd.actor import (  # noqa: E402
    M_CONV, MeasurementActor, conv_out, random_dqn_measurement)

PEAK_F32_MFMA = 157.3e12


def flops_per_env(L=5760, n_actions=21):
    macs, n = 0, L
    for ci, co, k, s in M_CONV:
        n = conv_out(n, k, s)
        macs += co * ci * k * n
    macs += 64 * n * 256 + 2 * 256 * 256 + 2 * 256 * n_actions
    return 2 * macs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--chunk", type=int, default=0)
    args = ap.parse_args()
    B, L = args.batch, 5760
    actor = MeasurementActor({k: v.cuda() for k, v in random_dqn_measurement(seed=1).items()}, read_length=L,
                             max_batch=B, seed=2, chunk=args.chunk)
    obs = torch.randn((B, 2, L), device="cuda") * 3
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
    fl = flops_per_env(L) * B
    print(json.dumps({"metric": "measurement-input DQN actor decisions/s (one qc_mactor_act over the batch)",
                      "value": B / ms * 1e3, "unit": "decisions/s", "batch": B, "ms_per_call": ms, "dtype": "f32",
                      "chunk": args.chunk or 2048,
                      "roofline": {"bound": "mfma", "achieved": fl / (ms * 1e-3) / 1e12,
                                   "peak": PEAK_F32_MFMA / 1e12, "unit": "TFLOP/s",
                                   "frac": fl / (ms * 1e-3) / PEAK_F32_MFMA, "flops_per_decision": flops_per_env(L)},
                      "note": "conv1..3 implicit GEMMs (buffer loads, split-K pairing) per env chunk + fc1 GEMM + noisy tail, in-kernel noise"}),
          flush=True)


if __name__ == "__main__":
    main()
