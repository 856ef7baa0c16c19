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
episode-return gather after the timed region. `--gpus N` under torchrun (WORLD_SIZE set) runs this rank;
without a launcher bench.py starts the N rank processes itself (before touching any GPU).
The k_step time in `roofline` comes from HIP events the library records around each k_step launch on
its stream (qc_set_timing); the CPU baseline runs the oracle in a child process on every usable host
core (oracle/cpu_bench.py).
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
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); without an external launcher bench.py starts them itself")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="metric")
    ap.add_argument("--batch", type=int, default=0, help="per-GPU batch (default: the config's)")
    ap.add_argument("--sub-steps", type=int, default=0, help="physics steps per bench step (default: control interval)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: every usable host core (affinity / cgroup quota)")
    ap.add_argument("--launch-timeout", type=float, default=0.0,
                    help="bench.py's own launcher: kill every rank after this many seconds (0: no limit)")
    ap.add_argument("--digest-envs", type=int, default=0,
                    help="report sha256 digests of the final state per run of this many envs (shard checks)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher check without a GPU: the ranks join a gloo group and report the world size")
    return ap.parse_args()


def launch_ranks(n: int, deadline_s: float = 0.0) -> int:
    """--gpus N without WORLD_SIZE in the environment: start N copies of this script as ranks 0..N-1
    (LOCAL_RANK = rank, one GPU each), before this process touches any GPU. Rank 0 prints the JSON line.
    The ranks are polled together (IHO/main_parallel.py:345-359 starts its workers the same way and would
    otherwise wait on a dead one forever): the first rank to exit non-zero has its siblings killed, its
    stderr tail repeated and its code returned, so a rank that dies in RCCL init ends the job in seconds
    instead of leaving the others blocked in the rendezvous. deadline_s > 0 bounds the whole job the same
    way (code 124). The driver's torchrun launch sets WORLD_SIZE and skips this."""
    import collections
    import socket
    import subprocess
    import threading
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs, tails, pumps = [], [], []

    def pump(stream, tail):
        # forward the rank's stderr line by line and keep its last lines for the failure report
        for line in iter(stream.readline, b""):
            tail.append(line.decode(errors="replace"))
            sys.stderr.write(line.decode(errors="replace"))
            sys.stderr.flush()
        stream.close()

    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        p = subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                             stderr=subprocess.PIPE)
        tail = collections.deque(maxlen=40)
        th = threading.Thread(target=pump, args=(p.stderr, tail), daemon=True)
        th.start()
        procs.append(p)
        tails.append(tail)
        pumps.append(th)

    def code_of(rc):
        return rc if rc >= 0 else 128 - rc       # killed by signal s: the shell's 128 + s

    t0 = time.monotonic()
    failed, rc_fail = None, 0
    while True:
        live = [p for p in procs if p.poll() is None]
        bad = [r for r, p in enumerate(procs) if p.returncode not in (None, 0)]
        if bad:
            failed = bad[0]
            rc_fail = code_of(procs[failed].returncode)
            break
        if not live:
            break
        if deadline_s and time.monotonic() - t0 > deadline_s:
            failed, rc_fail = -1, 124
            break
        time.sleep(0.05)
    if failed is not None:
        for p in procs:
            if p.poll() is None:
                p.kill()
        for p in procs:
            p.wait()
    for th in pumps:
        th.join(timeout=5)
    if failed is None:
        return 0
    if failed < 0:
        sys.stderr.write(f"bench.py: ranks still running after {deadline_s:.0f} s; all ranks killed\n")
    else:
        sys.stderr.write(f"bench.py: rank {failed} of {n} exited with code {rc_fail}; the other ranks were "
                         f"killed. Its stderr tail:\n" + "".join(tails[failed]))
    sys.stderr.flush()
    return rc_fail


def cpu_baseline(config: str, seconds: float, threads: int):
    """The oracle (CPU restatement of the reference scheme) on a bounded sample of the same workload, in a
    child process of its own (oracle/cpu_bench.py) so its OpenMP runtime starts with OMP_PROC_BIND=close
    on every usable host core."""
    import subprocess
    env = dict(os.environ, OMP_PROC_BIND="close", OMP_PLACES="cores")
    env.pop("OMP_NUM_THREADS", None)
    cmd = [sys.executable, "-m", "oracle.cpu_bench", "--config", config, "--seconds", str(seconds)]
    if threads:
        cmd += ["--threads", str(threads)]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=seconds * 4 + 120)
    if out.returncode != 0:
        raise RuntimeError(out.stderr[-2000:])
    return json.loads(out.stdout.strip().splitlines()[-1])


def lib_sha() -> str:
    """sha256 (16 hex digits) of the libqcart.so this run loads: a committed profile's traffic is only
    reported for the exact library it was measured on."""
    import hashlib
    from deepreinforcementlearningcontrolofquantumcartpoles_amd import _lib
    with open(_lib.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def latest_profile(workload: str, sha: str):
    """The newest committed rocprofv3 summary (profiles/*_summary.json, tools/prof_summary.py) whose
    profiled bench line ran this workload on this same library build and whose kernel is a k_step."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_summary.json"))):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        bl = d.get("bench_line") or {}
        if (bl.get("config", {}).get("workload") == workload and "hbm_bytes_per_launch" in d
                and bl.get("roofline", {}).get("lib_sha") == sha and "k_step" in d.get("kernel", "")):
            best = d
    return best


def latest_sq(workload: str, sha: str):
    """The newest committed SQ instruction-mix summary (profiles/*_sq.json, tools/sq_summary.py) of this
    workload on this same library build, or None."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_sq.json"))):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if d.get("workload") == workload and d.get("lib_sha") == sha:
            best = d
    return best


def executed_flops_per_elem(sq: dict, fp32: bool):
    """Executed floating-point operations per state element and env-step, from the SQ counters of the same
    library on the same workload: SQ_INSTS_VALU_FLOPS_FP64 / _FP32 count the flops of each wave instruction
    per lane (an FMA 2, a packed v_pk_fma_f32 4; the fp64 counter equals 2 FMA + MUL + ADD of the instruction
    counts exactly), x 64 lanes / N rows. Without those counters: fp64 from the FMA / MUL / ADD instruction
    counts; fp32 None (a packed instruction counts once there)."""
    d, N = sq.get("derived", {}), sq["N"]
    f = d.get("fp32_flops_counter_per_wave_step" if fp32 else "fp64_flops_counter_per_wave_step")
    if f:
        return 64.0 * f / N
    if not fp32 and d.get("f64_flops_per_wave_step_from_insts"):
        return d["f64_flops_per_wave_step_from_insts"] / N
    return None


def dry_run(world: int, rank: int):
    import torch
    import torch.distributed as dist
    if world > 1:
        from deepreinforcementlearningcontrolofquantumcartpoles_amd import distributed as D
        D.init_from_env("gloo")
    t = torch.ones(1)
    if world > 1:
        dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "world_size_seen": int(t.item())}), flush=True)
    if world > 1:
        dist.destroy_process_group()


M32 = 0xFFFFFFFF


def _hash32(x):
    """A 32-bit integer mix (two xorshift-multiply rounds) on an int64 tensor of values < 2^32; every
    intermediate product stays below 2^63."""
    x = ((x >> 16) ^ x) * 0x45D9F3B & M32
    x = ((x >> 16) ^ x) * 0x45D9F3B & M32
    return (x >> 16) ^ x


def synth_inputs(n_ctrl: int, B: int, offset: int, n_actions: int, dev):
    """Synthetic actions [n_ctrl][B] ~ U{0..n_actions-1} and Gaussian-packet parameters, keyed by the GLOBAL
    env id (offset + e) and the control step, so a rank's shard sees exactly the inputs of the same envs in a
    one-rank run of the whole batch (the Philox noise and psi0 are keyed the same way: env_offset)."""
    import torch
    gid = torch.arange(offset, offset + B, dtype=torch.int64, device=dev)
    k = torch.arange(n_ctrl, dtype=torch.int64, device=dev)
    x = (gid[None, :] * 0x9E3779B1 + k[:, None] * 0x85EBCA6B + 0x2545F491) & M32
    acts = (_hash32(x) % n_actions).to(torch.int32)

    def uniform(salt):
        return _hash32((gid * 0x9E3779B1 + salt) & M32).to(torch.float64) * 2.0 ** -32

    return acts.contiguous(), uniform(0x68E31DA4), uniform(0xB5297A4D), uniform(0x1B56C4E9)


def psi_digests(psi, chunk: int):
    """sha256 (16 hex digits) of the state's bytes per run of `chunk` envs, in env order."""
    import hashlib
    h = psi.cpu().contiguous().numpy()
    return [hashlib.sha256(h[i:i + chunk].tobytes()).hexdigest()[:16] for i in range(0, h.shape[0], chunk)]


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "0") or 0)
    # under a launcher (WORLD_SIZE set, world 1 included) the ranks form an RCCL group; a plain
    # `python bench.py` (N = 1) runs without one
    use_dist = world > 0
    if world == 0:
        if args.gpus > 1:
            sys.exit(launch_ranks(args.gpus, args.launch_timeout))
        world = 1
    elif world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # fault injection for the launcher tests: this rank exits at once with code 3 (or hangs)
    if os.environ.get("QCART_BENCH_FAIL_RANK", "") == str(rank):
        sys.stderr.write(f"bench.py rank {rank}: QCART_BENCH_FAIL_RANK, exiting with 3\n")
        sys.exit(3)
    if os.environ.get("QCART_BENCH_HANG_RANK", "") == str(rank):
        time.sleep(3600)
    if args.dry_run:
        return dry_run(world, rank)
    # rehearsal of the N-rank path on a one-GPU lease: every rank steps its shard on device 0 and gloo carries
    # the collectives (RCCL refuses two ranks on one device); timing, sharding and gathers are the N-GPU job's
    share = os.environ.get("QCART_BENCH_SHARE_DEVICE", "0") == "1"

    import torch
    import torch.distributed as dist

    from deepreinforcementlearningcontrolofquantumcartpoles_amd import config as cfg
    from deepreinforcementlearningcontrolofquantumcartpoles_amd import distributed as D
    from deepreinforcementlearningcontrolofquantumcartpoles_amd.core import Stepper

    if use_dist and share:
        torch.cuda.set_device(0)
        D.init_from_env("gloo")
    elif use_dist:
        D.init_from_env("nccl")              # RCCL (torch.distributed "nccl" on ROCm), one rank per GPU
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local if (use_dist and not share) else 0)

    def coll(x):
        # gloo (the rehearsal) takes host tensors
        return x.cpu() if share else x

    conf = cfg.BENCH_CONFIGS[args.config]
    ph = conf["physics"]
    B = args.batch or conf["batch"]
    n_sub = args.sub_steps or ph.control_interval
    st = Stepper(ph, B, dev, seed=42, env_offset=rank * B)
    psi = st.new_state()
    acts_all, u0, u1, u2 = synth_inputs(args.steps + args.warmup, B, rank * B, ph.n_actions, dev)
    if ph.fock:
        st.reset(psi, 1, arg0=16)       # synthetic psi0: random amplitudes on levels < 16
    else:
        st.reset(psi, 2, k=u0 * 0.6 - 0.3, mean=u1 * 2 - 1, std=u2 * 0.6 + 0.7)

    def one(k):
        return st.step(psi, acts_all[k], n_sub, want_fail=True, want_obs=True, want_term=(ph.family == 3))

    for k in range(args.warmup):
        one(k)
    torch.cuda.synchronize(dev)
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    st.set_timing(True)          # HIP events around each k_step launch, on the stream it runs on
    t0 = time.perf_counter()
    for k in range(args.steps):
        out = one(args.warmup + k)
    torch.cuda.synchronize(dev)
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    kern_total, launches = st.step_kernel_time()
    st.set_timing(False)
    kern_ms = kern_total / max(launches, 1)
    t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
    world_seen = 1
    rccl = None
    digests = psi_digests(psi, args.digest_envs) if args.digest_envs else None
    if use_dist:
        t = coll(t)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        world_seen = dist.get_world_size()
        # RCCL gather of per-env episode statistics after the timed region (distributed.gather_episode_stats,
        # device tensors): each env's survival through the last control step and its first Fail step
        survived = (out["fail_step"] == 0).to(torch.float64)
        R, L = D.gather_episode_stats(coll(survived), coll(out["fail_step"].to(torch.float64)))
        rccl = {"backend": dist.get_backend(), "world_size": world_seen, "gathered_envs": int(R.numel()),
                "gathered_survivors": float(R.sum().item()), "device": str(R.device), "share_device": share}
        if digests is not None:
            every = [None] * world_seen
            dist.all_gather_object(every, digests)
            digests = [d for r in every for d in r]
    elapsed, kern_ms = float(t[0]), float(t[1])
    sha = lib_sha()
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
        "config": {"workload": f"{cfg.FAMILY_NAMES[ph.family]} N={N} per-GPU batch={B} dt=1/{ph.time_steps} "
                               f"{n_sub} physics steps + moments per step ({args.config})",
                   "global_batch": B * world, "seq_len": N, "parallelism": f"env-shard{world}",
                   "physics_steps_per_step": n_sub, "world_size_seen": world_seen, "rccl": rccl},
        "psi_digests": digests,
        # bound / achieved / peak / frac: the north-star HBM yardstick — algorithmic psi bytes (read + write
        # per physics step) per k_step launch / the launch's time, against the HBM peak. What actually binds
        # k_step is the FP vector pipe (psi stays in VGPRs across the fused steps): that roofline is the
        # separate "binding" object, in TFLOP/s against the FP64 (FP32 for C5) vector peak
        "roofline": {"bound": "hbm", "achieved": achieved / 1e9, "peak": PEAK_HBM / 1e9, "unit": "GB/s",
                     "frac": achieved / PEAK_HBM, "traffic": None,
                     # "bound" is the north-star yardstick's (algorithmic psi bytes vs HBM peak); the pipe that
                     # actually limits k_step is "limiter" (= binding.bound)
                     "limiter": "fp32_valu" if fp32 else "fp64_valu",
                     "yardstick": f"{int(bpe)}*N B/env-step (psi read+write) x env-steps per launch / k_step time "
                                  "(SURVEY §8d north-star yardstick; the kernel keeps psi on chip, measured_gbs is "
                                  "the real HBM traffic rate)",
                     "kernel": "k_step", "kernel_ms": kern_ms, "kernel_launches": launches,
                     "lib_sha": sha,
                     "binding": {"bound": "fp32_valu" if fp32 else "fp64_valu", "achieved": flops / 1e12,
                                 "peak": peak_valu / 1e12, "unit": "TFLOP/s", "frac": flops / peak_valu,
                                 "flops_per_elem": FLOPS_PER_ELEM[ph.family]}},
        "rl_steps_per_s": value / ph.control_interval,
    }
    # HBM traffic per launch measured by rocprofv3 PMC (FETCH_SIZE x2 + WRITE_SIZE, tools/prof_summary.py)
    # for this same workload, when a committed profile exists
    prof = latest_profile(res["config"]["workload"], sha)
    if prof is not None:
        res["roofline"]["traffic"] = prof["hbm_bytes_per_launch"]
        res["roofline"]["traffic_unit"] = "bytes/launch (rocprofv3 PMC, profiles/%s_summary.json)" % prof["tag"]
        res["roofline"]["algorithmic_bytes_per_launch"] = bpe * N * per_launch_units
        res["roofline"]["measured_gbs"] = prof["hbm_bytes_per_launch"] / (kern_ms * 1e-3) / 1e9
    # the executed-flop count of the same library on this workload (rocprofv3 SQ counters), beside the nominal
    # per-element count of SURVEY §8d
    b = res["roofline"]["binding"]
    b["executed_flops_per_elem"] = b["executed_frac"] = b["executed_achieved"] = None
    sq = latest_sq(res["config"]["workload"], sha)
    if sq is not None:
        fe = executed_flops_per_elem(sq, fp32)
        if fe:
            ex = fe * N * per_launch_units / (kern_ms * 1e-3)
            b.update(executed_flops_per_elem=fe, executed_achieved=ex / 1e12, executed_frac=ex / peak_valu,
                     executed_source="profiles/%s_sq.json" % sq["tag"])
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            res["cpu_baseline"] = cpu_baseline(args.config, args.cpu_seconds, args.cpu_threads)
        except Exception as e:  # the baseline is reported, never fatal
            res["cpu_baseline"] = {"value": None, "error": repr(e)}
    if rank == 0:
        print(json.dumps(res), flush=True)
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
