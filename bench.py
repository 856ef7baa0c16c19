#!/usr/bin/env python3
"""Benchmark of the quantum-cartpole env.step() hot path (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config metric]

One bench "step" = one RL control step of the whole batch: every env advances one control
interval (80 physics steps for the IHO, IHO/main_parallel.py:113-118) with its own discrete action,
then the 5-moment observation is reduced (env.step() = propagation + observation). Inputs are
synthetic (random psi0 on Fock levels < 16, actions ~ U{0..20} redrawn every control step) and
resident in HBM before timing starts. value = physics env-steps/s over all ranks (one env-step =
one reference simulation.step call). Multi-GPU: one process per GPU, env shard per rank
(weak scaling, no data-path collective); RCCL all_reduce/all_gather only for the timing max and the
episode-return gather after the timed region.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# algorithmic flops per env-step per state element (recount in DESIGN.md §Roofline)
FLOPS_PER_ELEM = {0: 350, 1: 470, 2: 705, 3: 705}
PEAK_HBM = 8.0e12          # MI355X_MICROARCH.md: HBM3E 8 TB/s (spec)
PEAK_FP64_VALU = 78.6e12   # MI355X FP64 vector (spec)
PEAK_FP32_VALU = 157.3e12  # MI355X FP32 vector (spec; config C5 computes in fp32)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="metric")
    ap.add_argument("--batch", type=int, default=0, help="per-GPU batch (default: the config's)")
    ap.add_argument("--sub-steps", type=int, default=0, help="physics steps per bench step (default: control interval)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "16") or 16))
    return ap.parse_args()


def cpu_baseline(physics, seconds: float, threads: int):
    """The oracle (CPU restatement of the reference scheme) on a bounded sample of the same workload."""
    import numpy as np

    from oracle import oracle as O
    O.build()
    s = O.OracleSystem(physics.family, n_max=physics.n_max, omega=physics.omega, x_max=physics.x_max,
                       grid_size=physics.grid_size, lambda_=physics.lambda_, mass=physics.mass,
                       moment_order=physics.moment_order, a_mode=physics.a_mode)
    B = max(threads, 1) * 2
    psi = np.stack([s.fock_random_state(1234, e, 16) for e in range(B)]) if physics.fock else None
    if psi is None:
        rng = np.random.default_rng(1)
        psi = np.stack([s.gaussian_packet(rng.uniform(-.3, .3), rng.uniform(-1, 1), rng.uniform(.7, 1.3))
                        for _ in range(B)])
    acts = np.random.default_rng(0).integers(0, 21, B).astype(np.int32)
    s.run_batch(psi, acts, physics.f_max, 5, physics.dt, physics.gamma, seed=42, n_threads=threads)  # warm
    n = 0
    t0 = time.perf_counter()
    chunk = 20
    while time.perf_counter() - t0 < seconds:
        s.run_batch(psi, acts, physics.f_max, chunk, physics.dt, physics.gamma, seed=42, step0=n,
                    n_threads=threads)
        n += chunk
    dtm = time.perf_counter() - t0
    # single-core rate (one env on one thread, the reference's one-env-per-process model)
    one = psi[:1].copy()
    n1 = 0
    t1 = time.perf_counter()
    while time.perf_counter() - t1 < min(3.0, seconds / 4):
        s.run_batch(one, acts[:1], physics.f_max, chunk, physics.dt, physics.gamma, seed=42, step0=n1, n_threads=1)
        n1 += chunk
    d1 = time.perf_counter() - t1
    return {"value": B * n / dtm, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"{B} envs x {n} physics steps (N={physics.dim}, fp64, OpenMP over envs, "
                      f"one single-threaded env per thread), {dtm:.1f} s wall",
            "single_core_value": n1 / d1, "cpu_model": _cpu_model()}


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def latest_profile(workload: str):
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_summary.json"))):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        bl = d.get("bench_line") or {}
        if bl.get("config", {}).get("workload") == workload and "hbm_bytes_per_launch" in d:
            best = d
    return best


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from deepreinforcementlearningcontrolofquantumcartpoles_amd import config as cfg
    from deepreinforcementlearningcontrolofquantumcartpoles_amd.core import Stepper

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local if world > 1 else 0)

    conf = cfg.BENCH_CONFIGS[args.config]
    ph = conf["physics"]
    B = args.batch or conf["batch"]
    n_sub = args.sub_steps or ph.control_interval
    st = Stepper(ph, B, dev, seed=42, env_offset=rank * B)
    psi = st.new_state()
    if ph.fock:
        st.reset(psi, 1, arg0=16)       # synthetic psi0: random amplitudes on levels < 16
    else:
        g = torch.Generator(device="cpu").manual_seed(1234 + rank)
        k = (torch.rand(B, generator=g, dtype=torch.float64) * 0.6 - 0.3).to(dev)
        mu = (torch.rand(B, generator=g, dtype=torch.float64) * 2 - 1).to(dev)
        sg = (torch.rand(B, generator=g, dtype=torch.float64) * 0.6 + 0.7).to(dev)
        st.reset(psi, 2, k=k, mean=mu, std=sg)
    gen = torch.Generator(device=dev).manual_seed(7 + rank)
    acts_all = torch.randint(0, ph.n_actions, (args.steps + args.warmup, B), generator=gen, device=dev,
                             dtype=torch.int32)
    stream = torch.cuda.current_stream(dev)

    def one(k):
        return st.step(psi, acts_all[k], n_sub, want_fail=True, want_obs=True, want_term=(ph.family == 3))

    for k in range(args.warmup):
        one(k)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        evs[k][0].record(stream)
        out = one(args.warmup + k)
        evs[k][1].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    kern_ms = sum(a.elapsed_time(b) for a, b in evs) / args.steps
    t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        # RCCL gather of per-env episode statistics (here: survival flags of this control step)
        alive = (out["fail_step"] == 0).to(torch.float64).sum().reshape(1)
        gathered = [torch.zeros_like(alive) for _ in range(world)]
        dist.all_gather(gathered, alive)
    elapsed, kern_ms = float(t[0]), float(t[1])
    units = B * world * n_sub * args.steps
    value = units / elapsed
    N = ph.dim
    per_launch_units = B * n_sub
    fp32 = ph.precision == 1
    bpe = 16.0 if fp32 else 32.0             # psi read + write per element: complex64 / complex128
    peak_valu = PEAK_FP32_VALU if fp32 else PEAK_FP64_VALU
    achieved = bpe * N * per_launch_units / (kern_ms * 1e-3)
    flops = FLOPS_PER_ELEM[ph.family] * N * per_launch_units / (kern_ms * 1e-3)
    res = {
        "metric": "env-steps/sec (whole node), inverted-harmonic grid=512 batch=65536; 1/2/4/8 GPU",
        "value": value,
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32" if fp32 else "f64",
        "data": ("synthetic (random psi0 on Fock levels < 16; actions ~ U{0..20} per control step)" if ph.fock else
                 "synthetic (Gaussian packets mu~U[-1,1], sigma~U[0.7,1.3], k~U[-0.3,0.3]; actions ~ U{0..20} "
                 "per control step)"),
        "config": {"workload": f"{cfg.FAMILY_NAMES[ph.family]} N={N} per-GPU batch={B} "
                               f"{n_sub} physics steps + moments per step ({args.config})",
                   "global_batch": B * world, "seq_len": N, "parallelism": f"env-shard{world}",
                   "physics_steps_per_step": n_sub},
        "roofline": {"bound": "hbm", "achieved": achieved / 1e9, "peak": PEAK_HBM / 1e9, "unit": "GB/s",
                     "frac": achieved / PEAK_HBM, "traffic": None,
                     "kernel": "k_step", "kernel_ms": kern_ms,
                     "note": f"achieved = {int(bpe)}*N B/env-step (psi read+write) x env-steps per launch / launch time"},
        "rl_steps_per_s": value / ph.control_interval,
        "valu": {"achieved_tflops": flops / 1e12, "peak_tflops": peak_valu / 1e12,
                 "frac": flops / peak_valu, "flops_per_elem": FLOPS_PER_ELEM[ph.family]},
    }
    # HBM traffic per launch measured by rocprofv3 PMC (FETCH_SIZE x2 + WRITE_SIZE, tools/prof_summary.py)
    # for this same workload, when a committed profile exists
    prof = latest_profile(res["config"]["workload"])
    if prof is not None:
        res["roofline"]["traffic"] = prof["hbm_bytes_per_launch"]
        res["roofline"]["traffic_unit"] = "bytes/launch (rocprofv3 PMC, profiles/%s_summary.json)" % prof["tag"]
        res["roofline"]["algorithmic_bytes_per_launch"] = bpe * N * per_launch_units
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            res["cpu_baseline"] = cpu_baseline(ph, args.cpu_seconds, args.cpu_threads)
        except Exception as e:  # the baseline is reported, never fatal
            res["cpu_baseline"] = {"value": None, "error": repr(e)}
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
