"""Throughput of the drop-in `simulation` module (B = 1, numpy state, one kernel launch and two host
copies per call): the reference drivers' own call pattern, IHO/main_parallel.py:264.

    python tools/bench_dropin.py [--n-max 180] [--calls 2000]
    python tools/bench_dropin.py --procs 1,8,16 [--seconds 5] [--n-max 180] [--kinds gpu,cpu] [--out FILE]

--procs: the reference's process model (IHO/main_parallel.py:345-359: 30-40 actor processes, each with its
own `simulation` module stepping one env): P independent processes, each `install()`ing the drop-in and calling
`step` on one env, started together behind a file barrier. Kinds:
  gpu     each process its own plain drop-in (its own HIP context, B = 1 launches, copies and syncs per call)
  server  one StepServer process owns the GPU (qc_server_*); the P processes attach with
          install(..., server=name) (libqcart_client.so, no HIP in them) and every tick steps all pending envs in
          one batched launch
  cpu     the oracle (the CPU restatement, one env and one host core each — what the reference's processes do)
The aggregate counts every process's step calls inside the COMMON window [latest start, earliest end] (each
process records its call count after every control interval; counts at the window edges interpolated) divided by
that window. The parent never touches the GPU; each process is a fresh child.

--family (default inverted_harmonic): any of the four modules at its driver defaults (config.DEFAULTS; --n-max for the
Fock ones): dt, gamma and the action grid's forces of that driver, one control interval per force (IHO 80 steps, IQO
160), the episode restarted after each from |0> (Fock) or the drivers' Gaussian packet (grid). --driver-loop adds the
driver's per-interval call: x_expectation (IHO/main_parallel.py:246) or get_moments (IQO/main_parallel.py:134,202).
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time
from math import pi

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def single(args):
    from deepreinforcementlearningcontrolofquantumcartpoles_amd import config as cfg
    from deepreinforcementlearningcontrolofquantumcartpoles_amd import simulation as S
    sim = S.load(cfg.IHO, n_max=args.n_max)
    sim.set_seed(1)
    state = np.zeros(args.n_max + 1, np.complex128)
    state[0] = 1.0
    dt, gamma = 1 / 1440, 2 * pi
    for _ in range(50):
        sim.step(state, dt, 0.0, gamma)
    out = {}
    for name, fn, per in (("step", sim.step, 1), ("simulate_10_steps", sim.simulate_10_steps, 10)):
        n = args.calls // per
        t0 = time.perf_counter()
        for k in range(n):
            fn(state, dt, 0.8 * ((k // 80) % 3 - 1), gamma)
        dtm = time.perf_counter() - t0
        out[name] = {"calls_per_s": n / dtm, "env_steps_per_s": n * per / dtm, "us_per_call": dtm / n * 1e6}
    print(json.dumps({"n_max": args.n_max, **out}))


def physics(args):
    from deepreinforcementlearningcontrolofquantumcartpoles_amd import config as cfg
    fam = {v: k for k, v in cfg.FAMILY_NAMES.items()}[args.family]
    ph = cfg.DEFAULTS[fam]
    return ph.with_(n_max=args.n_max) if ph.fock else ph


def initial_state(ph):
    """|0> (Fock) or the grid drivers' Gaussian packet (mean 0, std 1, IQO/main_parallel.py:182-183)."""
    if ph.fock:
        st = np.zeros(ph.dim, np.complex128)
        st[0] = 1.0
        return st
    x = (np.arange(ph.dim) - ph.dim // 2) * ph.grid_size
    st = np.exp(-x * x / 4.0).astype(np.complex128)
    return st / np.linalg.norm(st)


def worker(args):
    """One actor process: the drivers' call sequence (install, set_seed, step per dt; a force of the action grid per
    control interval) on one env, timed after the go file appears."""
    ph = physics(args)
    dt, gamma, ci = ph.dt, ph.gamma, ph.control_interval
    half = ph.n_actions // 2
    state = initial_state(ph)
    fresh = state.copy()
    obs = np.zeros(ph.n_obs)
    if args.kind in ("gpu", "server"):
        from deepreinforcementlearningcontrolofquantumcartpoles_amd import simulation as S
        kw = {"n_max": args.n_max} if ph.fock else {}
        sim = S.install(args.family, device=0, server=args.name if args.kind == "server" else None, **kw)
        sim.set_seed(1000 + args.rank)

        def step(F):
            return sim.step(state, dt, F, gamma)

        def per_interval():
            return sim.x_expectation(state) if ph.fock else sim.get_moments(state, obs)
    else:
        from oracle import oracle as O
        o = O.OracleSystem(ph.family, n_max=ph.n_max, omega=ph.omega, x_max=ph.x_max, grid_size=ph.grid_size,
                           lambda_=ph.lambda_, mass=ph.mass, moment_order=ph.moment_order)
        mt = O.MT19937(1000 + args.rank)

        def step(F):
            return o.step(state, dt, F, gamma, mt.normals(2))

        def per_interval():
            return o.x_expectation(state) if ph.fock else o.moments(state)

    def force(n):
        return ph.force(half + (n // ci) % 3 - 1)
    for k in range(3 * ci):                          # warm-up (tables of the forces used below)
        step(force(k))
        if k % ci == ci - 1:
            state[:] = fresh
    print("ready", flush=True)
    while not os.path.exists(args.go):
        time.sleep(0.001)
    n = 0
    t0 = time.time()
    t_end = t0 + args.seconds
    marks = [(t0, 0)]
    while True:
        for _ in range(ci):                            # one control interval per force
            step(force(n))
            n += 1
        if args.driver_loop:                           # the driver's own call per control interval
            per_interval()
        state[:] = fresh                               # restart the episode (keeps the env physical)
        t = time.time()
        marks.append((t, n))
        if t >= t_end:
            break
    print(json.dumps({"rank": args.rank, "calls": n, "t0": t0, "t1": t, "marks": marks}), flush=True)


def serve(args):
    """The step-server process: owns the GPU, serves until its stdin closes, prints its statistics."""
    import threading
    from deepreinforcementlearningcontrolofquantumcartpoles_amd import simulation as S
    kw = {"n_max": args.n_max} if physics(args).fock else {}
    srv = S.StepServer(args.family, max_clients=args.max_clients, name=args.name, device=0,
                       batch_wait_us=args.batch_wait_us, **kw)

    def watch():
        sys.stdin.read()
        srv.stop()
    threading.Thread(target=watch, daemon=True).start()
    print("ready", flush=True)
    srv.run(0)
    print(json.dumps(srv.stats()), flush=True)
    srv.close()


def cpu_stat():
    """The cgroup's CPU-quota throttling counters (cgroup v2 cpu.stat; {} where absent): P spinning processes over
    a CPU quota stall together for the rest of the quota period."""
    try:
        return {k: int(v) for k, v in (l.split() for l in open("/sys/fs/cgroup/cpu.stat"))}
    except (OSError, ValueError):
        return {}


def fan_out(args, kind, P):
    go = os.path.join(tempfile.mkdtemp(prefix="qcart_dropin_"), "go")
    env = dict(os.environ, OMP_NUM_THREADS="1", MKL_NUM_THREADS="1")
    server = None
    name = f"/qcart_bench_{os.getpid()}_{P}"
    if kind == "server":
        serr = open(go + ".server_err", "w+")
        cmd = [sys.executable, os.path.abspath(__file__), "--serve", "--name", name, "--max-clients", str(P),
               "--n-max", str(args.n_max), "--batch-wait-us", str(args.batch_wait_us), "--family", args.family]
        if args.server_prof:   # the server under rocprofv3 (kernel + HIP API trace: tools/server_timeline.py)
            cmd = ["rocprofv3", "--kernel-trace", "--hip-trace", "--output-format", "csv", "-d",
                   os.path.abspath(args.server_prof), "-o", "run", "--"] + cmd
        server = subprocess.Popen(cmd, cwd=ROOT, env=dict(env, TMPDIR="/tmp") if args.server_prof else env, stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=serr,
                                  text=True)
        if not server.stdout.readline().startswith("ready"):
            server.wait()
            serr.seek(0)
            raise RuntimeError(serr.read()[-2000:])
    errs = [open(go + f".err{r}", "w+") for r in range(P)]
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--worker", "--kind", kind, "--rank", str(r),
                               "--go", go, "--seconds", str(args.seconds), "--n-max", str(args.n_max),
                               "--name", name, "--family", args.family] + (["--driver-loop"] if args.driver_loop else []),
                              cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=errs[r], text=True)
             for r in range(P)]

    def fail(r):
        for p in procs + ([server] if server else []):
            if p.poll() is None:
                p.kill()
        errs[r].seek(0)
        raise RuntimeError(errs[r].read()[-2000:])
    for r, p in enumerate(procs):                      # every process ready (module loaded, warmed up)
        if not p.stdout.readline().startswith("ready"):
            p.wait()
            fail(r)
    cs0 = cpu_stat()
    open(go, "w").close()
    res = []
    for r, p in enumerate(procs):
        out, _ = p.communicate(timeout=args.seconds * 4 + 120)
        if p.returncode != 0:
            fail(r)
        res.append(json.loads(out.strip().splitlines()[-1]))
    cs1 = cpu_stat()
    srv_stats = None
    if server is not None:
        out, _ = server.communicate(input="", timeout=120)
        srv_stats = json.loads(out.strip().splitlines()[-1])
    # the common window [latest start, earliest end]: every process was stepping throughout it; each process's
    # calls inside it from its per-interval marks (interpolated at the edges)
    import numpy as np
    T0, T1 = max(r["t0"] for r in res), min(r["t1"] for r in res)
    if T1 - T0 < 0.5 * args.seconds:
        raise RuntimeError(f"the processes overlapped only {T1 - T0:.2f} s of {args.seconds} s")
    inside = 0.0
    for r in res:
        t, n = np.array(r["marks"]).T
        inside += float(np.interp(T1, t, n) - np.interp(T0, t, n))
    agg = inside / (T1 - T0)
    row = {"kind": kind, "procs": P, "driver_loop": bool(args.driver_loop), "step_calls_per_s": agg,
           "per_proc_calls_per_s": agg / P,
           "us_per_call": P / agg * 1e6, "seconds": args.seconds, "common_window_s": T1 - T0}
    if cs0 and cs1:
        row["cgroup"] = {k: cs1[k] - cs0.get(k, 0) for k in ("nr_periods", "nr_throttled", "throttled_usec", "usage_usec")
                         if k in cs1}
    if srv_stats:
        row["server"] = dict(srv_stats, calls_per_tick=srv_stats["calls"] / max(1, srv_stats["ticks"]))
    return row


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-max", type=int, default=180)
    ap.add_argument("--calls", type=int, default=2000)
    ap.add_argument("--procs", default="")
    ap.add_argument("--seconds", type=float, default=5.0)
    ap.add_argument("--kinds", default="gpu", help="gpu,server,cpu: the plain drop-in / the step server / the oracle")
    ap.add_argument("--out", default="")
    ap.add_argument("--worker", action="store_true")
    ap.add_argument("--kind", default="gpu")
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--go", default="")
    ap.add_argument("--serve", action="store_true")
    ap.add_argument("--name", default="")
    ap.add_argument("--max-clients", type=int, default=16)
    ap.add_argument("--batch-wait-us", type=float, default=40.0)
    ap.add_argument("--family", default="inverted_harmonic", help="harmonic / inverted_harmonic / quartic / inverted_quartic")
    ap.add_argument("--driver-loop", action="store_true",
                    help="also the driver's per-interval call: x_expectation (IHO/main_parallel.py:246) / get_moments "
                         "(IQO/main_parallel.py:202)")
    ap.add_argument("--server-prof", default="", help="run the server under rocprofv3 kernel + HIP trace into DIR")
    args = ap.parse_args()
    if args.serve:
        return serve(args)
    if args.worker:
        return worker(args)
    if not args.procs:
        return single(args)
    rows = []
    for kind in args.kinds.split(","):
        for P in [int(x) for x in args.procs.split(",")]:
            r = fan_out(args, kind, P)
            print(json.dumps(r), flush=True)
            rows.append(r)
    ph = physics(args)
    res = {"family": args.family, "n_max": args.n_max if ph.fock else None, "dim": ph.dim,
           "call": f"simulation.step(state, 1/{ph.time_steps}, F, gamma) (the driver's defaults), F of the action grid "
                   f"redrawn every {ph.control_interval} steps",
           "model": "P independent actor processes, one env each (IHO/main_parallel.py:345-359)", "rows": rows}
    if args.out:
        json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
