"""CPU baseline of bench.py (BASELINE.md §2 / SURVEY §8d) — TEST INFRASTRUCTURE ONLY: the oracle (the CPU
restatement of the reference scheme) timed on the host cores, in a process of its own so that the
OpenMP runtime starts with OMP_PROC_BIND=close / OMP_PLACES=cores (bench.py runs it as a child; it
never touches the GPU).

    python -m oracle.cpu_bench --config metric --seconds 12 [--threads N]

Execution model (the reference's, IHO/main_parallel.py:345-359, HO/setupC.py:44): one single-threaded
env per thread, OpenMP over envs (2 envs per thread), the bench's synthetic inputs and random actions.
100 warm-up steps, then whole control-interval chunks until `seconds` have passed. Prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def visible_cores() -> dict:
    """Cores this process may use: the affinity mask, capped by a cgroup v2 CPU quota when one is set."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    usable = aff if quota is None else max(1, min(aff, int(math.floor(quota + 1e-9))))
    return {"affinity": aff, "cgroup_quota": quota, "usable": usable}


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="metric")
    ap.add_argument("--seconds", type=float, default=12.0)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--warmup", type=int, default=100)
    args = ap.parse_args()
    import numpy as np

    from deepreinforcementlearningcontrolofquantumcartpoles_amd import config as cfg
    from oracle import oracle as O

    conf = cfg.BENCH_CONFIGS[args.config]
    ph = conf["physics"]
    cores = visible_cores()
    # the sample is never wider than the config's own batch (C1 is one env: one env on one core)
    threads = min(args.threads or cores["usable"], conf["batch"])
    s = O.OracleSystem(ph.family, n_max=ph.n_max, omega=ph.omega, x_max=ph.x_max, grid_size=ph.grid_size,
                       lambda_=ph.lambda_, mass=ph.mass, moment_order=ph.moment_order, a_mode=ph.a_mode)
    B = min(2 * threads, conf["batch"])
    if ph.fock:
        psi = np.stack([s.fock_random_state(1234, e, 16) for e in range(B)])
    else:
        rng = np.random.default_rng(1)
        psi = np.stack([s.gaussian_packet(rng.uniform(-.3, .3), rng.uniform(-1, 1), rng.uniform(.7, 1.3))
                        for _ in range(B)])
        psi /= np.linalg.norm(psi, axis=1, keepdims=True) * math.sqrt(ph.grid_size)
    acts = np.random.default_rng(0).integers(0, 21, B).astype(np.int32)
    s.run_batch(psi, acts, ph.f_max, args.warmup, ph.dt, ph.gamma, seed=42, n_threads=threads)
    chunk = ph.control_interval
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < args.seconds:
        s.run_batch(psi, acts, ph.f_max, chunk, ph.dt, ph.gamma, seed=42, step0=args.warmup + n, n_threads=threads)
        n += chunk
    dt_all = time.perf_counter() - t0
    one = psi[:1].copy()
    n1 = 0
    t1 = time.perf_counter()
    while time.perf_counter() - t1 < min(3.0, args.seconds / 4):
        s.run_batch(one, acts[:1], ph.f_max, chunk, ph.dt, ph.gamma, seed=42, step0=n1, n_threads=1)
        n1 += chunk
    d1 = time.perf_counter() - t1
    print(json.dumps({
        "value": B * n / dt_all, "unit": "env-steps/s", "cores": threads, "kind": "port",
        "sample": (f"{B} envs x {n} physics steps after {args.warmup} warm-up steps (N={ph.dim}, fp64, OpenMP "
                   f"over envs with OMP_PROC_BIND={os.environ.get('OMP_PROC_BIND')}, one single-threaded env per "
                   f"thread), {dt_all:.1f} s wall"),
        "single_core_value": n1 / d1, "cpu_model": cpu_model(), "visible_cores": cores,
    }), flush=True)


if __name__ == "__main__":
    main()
