#!/usr/bin/env python3
"""The step server in one process (tools/bench_dropin.py --kinds server runs it across processes): a StepServer
thread and P client threads (one env each, the drivers' step call per dt, ctypes releases the GIL) for a few
seconds; prints the server's per-tick phase times. Run it under rocprofv3 --kernel-trace --stats to see the tick's
kernels. python3 tools/server_profile.py [--procs 16] [--seconds 2] [--n-max 511]"""
import argparse
import json
import os
import sys
import threading
import time
from math import pi

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from deepreinforcementlearningcontrolofquantumcartpoles_amd import config as cfg  # noqa: E402
from deepreinforcementlearningcontrolofquantumcartpoles_amd import simulation as S  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=16)
    ap.add_argument("--seconds", type=float, default=2.0)
    ap.add_argument("--n-max", type=int, default=511)
    a = ap.parse_args()
    name = f"/qcart_prof_{os.getpid()}"
    srv = S.StepServer(cfg.IHO, max_clients=a.procs, name=name, n_max=a.n_max).start()
    counts = [0] * a.procs
    t_end = time.time() + a.seconds

    def run(c):
        m = S._ServedSimulation(cfg.DEFAULTS[cfg.IHO].with_(n_max=a.n_max), name)
        m.set_seed(1000 + c)
        st = np.zeros(a.n_max + 1, np.complex128)
        st[0] = 1
        n = 0
        while time.time() < t_end:
            for _ in range(80):
                m.step(st, 1 / 1440, 0.8 * ((n // 80) % 3 - 1), 2 * pi)
                n += 1
            st[:] = 0
            st[0] = 1
        counts[c] = n
        m.close()
    ts = [threading.Thread(target=run, args=(c,)) for c in range(a.procs)]
    t0 = time.time()
    [t.start() for t in ts]
    [t.join() for t in ts]
    dt = time.time() - t0
    st = srv.stats()
    srv.close()
    print(json.dumps({"procs": a.procs, "calls_per_s": sum(counts) / dt, **st}))


if __name__ == "__main__":
    main()
