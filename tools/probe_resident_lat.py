"""One client's step() latency through the step server at the IHO driver's n_max = 180, on the resident kernel and
on the ticks (QCART_SERVER_RESIDENT=0, a server of its own): from C (tools/probe_resident_lat.c, no Python in the
call) and through the served Python module (the drivers' call), µs per call. The server runs in this process.
    python tools/probe_resident_lat.py [--calls 20000]
    QCART_LIB=.../libqcart_rstamp.so python tools/probe_resident_lat.py --stamps   (make expt EXPT=-DQCART_RES_STAMPS=1
        NAME=rstamp TU=qcart_k_iho: the resident wave's phase clocks, µs per request, from the C client's slot)"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def wave_phases(name):
    """The QCART_RES_STAMPS build's per-slot sums (slot 0: the C client's), µs per request: acquire, pair, step,
    results + release."""
    import ctypes
    import mmap
    from tests.test_server_protocol import Header, Slot
    with open("/dev/shm" + name, "rb") as f:
        mm = mmap.mmap(f.fileno(), 0, prot=mmap.PROT_READ)
        h = Header.from_buffer_copy(mm[:ctypes.sizeof(Header)])
        off = h.slot_off + Slot.err.offset
        v = [int.from_bytes(mm[off + 8 * i:off + 8 * i + 8], "little") for i in range(5)]
        mm.close()
    n = max(1, v[0])
    return {"requests": v[0], **{k: round(x / n * 0.01, 3) for k, x in zip(("acquire", "pair", "step", "publish"), v[1:])}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=20000)
    ap.add_argument("--n-max", type=int, default=180)
    ap.add_argument("--stamps", action="store_true")
    args = ap.parse_args()
    import numpy as np
    from deepreinforcementlearningcontrolofquantumcartpoles_amd import config as cfg
    from deepreinforcementlearningcontrolofquantumcartpoles_amd import simulation as S
    rows = []
    for mode in ("resident", "ticks"):
        if mode == "ticks":
            os.environ["QCART_SERVER_RESIDENT"] = "0"
        name = f"/qcart_lat_{os.getpid()}_{mode}"
        srv = S.StepServer(cfg.IHO, max_clients=2, name=name, n_max=args.n_max).start()
        try:
            out = subprocess.run([os.path.join(ROOT, "tools/bin/probe_resident_lat"), name, str(args.calls)],
                                 capture_output=True, text=True, timeout=120)
            c_row = json.loads(out.stdout) if out.returncode == 0 else {"error": out.stderr}
            if args.stamps and mode == "resident":
                c_row["phases_us"] = wave_phases(name)
            m = S._ServedSimulation(cfg.DEFAULTS[cfg.IHO].with_(n_max=args.n_max), name)
            st = np.zeros(args.n_max + 1, np.complex128)
            for k in range(args.calls + 200):
                if k % 80 == 0:
                    st[:] = 0
                    st[0] = 1
                if k == 200:
                    t0 = time.perf_counter()
                m.step(st, 1 / 1440, 0.8, 2 * np.pi)
            py_us = (time.perf_counter() - t0) / args.calls * 1e6
            m.close()
            stats = srv.stats()
        finally:
            srv.close()
        rows.append({"path": mode, "c_us_per_call": c_row.get("us_per_call"), "python_us_per_call": round(py_us, 2),
                     **({"wave_phases_us": c_row["phases_us"]} if "phases_us" in c_row else {}),
                     "resident": stats["resident"]})
        print(json.dumps(rows[-1]), flush=True)
    os.environ.pop("QCART_SERVER_RESIDENT", None)


if __name__ == "__main__":
    main()
