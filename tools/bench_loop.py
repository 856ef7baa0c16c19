#!/usr/bin/env python3
"""End-to-end actor loop on one GPU (SURVEY §8f rank 1 measured in place): BatchedEnv (IHO N = 512) +
DQNActor (direct_DQN, random-initialised weights of the reference architecture) for K control steps:
act -> step (80 physics steps) -> experience rows stored in the device prioritized replay (the drivers'
capacity 7000 x 18 x 100 = 12.6 M rows, qc_replay_store_xp) -> one sample(512) + batch_update, the
trainer's per-step memory traffic (RL.py:172, :224), with auto-reset of finished episodes.
With --input measurements: BatchedEnv(input='measurements') (the measurement record, qc_record) +
MeasurementActor (DQN_measurement) + the replay storing the reference's 5 915-float rows (capacity
--capacity rows; the drivers' 2.7 M-row memory is 64 GB, the bench default keeps 262 144 rows).
Prints one JSON line: RL steps/s (decisions), env-steps/s and the actor's / replay's share of the loop.
usage: python tools/bench_loop.py [--batch B] [--steps K] [--input xp|measurements]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from deepreinforcementlearningcontrolofquantumcartpoles_amd import config as cfg  # noqa: E402
from deepreinforcementlearningcontrolofquantumcartpoles_amd.actor import (  # noqa: E402
    DQNActor, MeasurementActor, random_direct_dqn, random_dqn_measurement)
from deepreinforcementlearningcontrolofquantumcartpoles_amd.env import BatchedEnv  # noqa: E402
from deepreinforcementlearningcontrolofquantumcartpoles_amd.replay import PrioritizedReplay  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=20)   # ~0.5 s: a fresh box ramps its clock over the first launches
    ap.add_argument("--capacity", type=int, default=0)   # xp: 7000 x 18 x 100 (IHO/arguments.py:80, main_parallel.py:595)
    ap.add_argument("--input", choices=("xp", "measurements"), default="xp")
    ap.add_argument("--reset", choices=("immediate", "deferred"), default=None,
                    help="BatchedEnv auto-reset mode (deferred: finished envs reset in the next call's launch, no host "
                         "sync; the default for 'xp', where it applies; immediate for 'measurements')")
    ap.add_argument("--marker", action="store_true",
                    help="wrap the timed steps in a roctx range 'timed' (tools/loop_breakdown.py, rocprofv3 --marker-trace)")
    args = ap.parse_args()
    if args.reset is None:
        args.reset = "deferred" if args.input == "xp" else "immediate"
    B = args.batch
    meas = args.input == "measurements"
    ph = cfg.DEFAULTS[cfg.IHO].with_(n_max=511)
    env = BatchedEnv(ph, B, 0, seed=1, input=args.input, reset=args.reset)
    if meas:
        actor = MeasurementActor({k: v.cuda() for k, v in random_dqn_measurement(seed=1).items()}, max_batch=B, seed=2)
        row_len = int(env.rows.shape[1])
        mem = PrioritizedReplay(args.capacity or 262144, row_len, "random", 0.2, device=0, seed=3)
    else:
        actor = DQNActor({k: v.cuda() for k, v in random_direct_dqn(seed=1).items()}, max_batch=B, seed=2)
        mem = PrioritizedReplay(args.capacity or 7000 * 18 * 100, 2 * 5 + 2, "random", 0.2, device=0, seed=3)
    obs = env.reset()
    steps_done = 0
    ev = lambda: torch.cuda.Event(enable_timing=True)   # noqa: E731
    marks = []                                          # (actor start, end, replay start, end) per timed step
    rows = torch.zeros((), dtype=torch.int64, device="cuda")
    n_done = torch.zeros((), dtype=torch.int64, device="cuda")
    # no host synchronisation inside the timed loop (device counters, events read afterwards): the loop's own
    # cost is what the GPU sees
    for it in range(args.warmup + args.steps):
        if it == args.warmup:
            torch.cuda.synchronize()
            if args.marker:
                torch.cuda.nvtx.range_push("timed")
            t0 = time.perf_counter()
            rows.zero_()
            n_done.zero_()
        m = [ev(), ev(), ev(), ev()]
        m[0].record()
        a = actor.act(obs, eps=DQNActor.eps_threshold(steps_done))
        m[1].record()
        steps_done += B
        obs, reward, done, info = env.step(a)
        rows += info["valid"].sum()
        n_done += done.sum()
        m[2].record()
        if meas:
            mem.store(info["rows"], info["valid"])
        else:
            # the row of a done env holds its terminal observation (IHO/main_parallel.py:250-257); in the immediate
            # mode the returned obs of a done env is already the next episode's
            nxt = torch.where(done[:, None], info["terminal_obs"], obs) if "terminal_obs" in info else obs
            mem.store_xp(info["last_obs"], nxt, a, reward, info["valid"])
        smp = mem.obtain_sample(512) if it > 0 else None
        if smp is not None:
            mem.batch_update(smp[0], torch.rand(512, device="cuda"))
        m[3].record()
        if it >= args.warmup:
            marks.append(m)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if args.marker:
        torch.cuda.nvtx.range_pop()
    actor_ms = sum(m[0].elapsed_time(m[1]) for m in marks)
    replay_ms = sum(m[2].elapsed_time(m[3]) for m in marks)
    rows = int(rows)
    done_frac = int(n_done) / (B * args.steps)
    K = args.steps
    net = "DQN_measurement" if meas else "direct_DQN"
    print(json.dumps({"metric": f"actor loop RL steps/s (BatchedEnv IHO N=512 input={args.input} reset={args.reset} + device {net} actor)",
                      "value": B * K / dt, "unit": "decisions/s", "env_steps_per_s": B * K * ph.control_interval / dt,
                      # physics env-steps actually taken: the immediate mode adds the reset intervals of the envs
                      # finished in each call (deferred: they are among the B per call)
                      "physics_env_steps_per_s": (B * K + (int(n_done) if args.reset == "immediate" else 0))
                      * ph.control_interval / dt,
                      "batch": B, "control_steps": K, "ms_per_control_step": dt / K * 1e3,
                      "actor_ms_per_control_step": actor_ms / K, "actor_share": actor_ms / (dt * 1e3),
                      "replay_ms_per_control_step": replay_ms / K, "replay_share": replay_ms / (dt * 1e3),
                      "replay_len": len(mem),
                      "done_fraction_per_control_step": done_frac,
                      "experience_rows_per_s": rows / dt,
                      "row_len": mem.data_size,
                      "data": f"synthetic: |0> resets, random-initialised {net} weights"}), flush=True)


if __name__ == "__main__":
    main()
