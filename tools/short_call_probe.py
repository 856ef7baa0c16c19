#!/usr/bin/env python3
"""Where a short step call's time goes: B envs (the step server's tick, the drop-in's call), one physics step per
call, with ψ / actions / step budgets either in device memory or in pinned, device-mapped host memory (the
server's placement: the clients' registered shm rows and mapped tick arrays). Run under rocprofv3 --kernel-trace
--stats per variant for the kernel's own duration; prints the host-timed call (launch + kernel + sync).
    python3 tools/short_call_probe.py --variant {dev,psi_host,all_host,arrays_host} [--batch 16] [--calls 500]"""
import argparse
import ctypes
import json
import os
import sys
import time
from math import pi

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deepreinforcementlearningcontrolofquantumcartpoles_amd import _lib as L  # noqa: E402
from deepreinforcementlearningcontrolofquantumcartpoles_amd import config as cfg  # noqa: E402
from deepreinforcementlearningcontrolofquantumcartpoles_amd.core import Stepper  # noqa: E402

HIP = ctypes.CDLL("libamdhip64.so")


def mapped(nbytes):
    """hipHostMalloc(hipHostMallocMapped) + its device pointer"""
    h = ctypes.c_void_p()
    assert HIP.hipHostMalloc(ctypes.byref(h), ctypes.c_size_t(nbytes), ctypes.c_uint(2)) == 0
    d = ctypes.c_void_p()
    assert HIP.hipHostGetDevicePointer(ctypes.byref(d), h, ctypes.c_uint(0)) == 0
    ctypes.memset(h, 0, nbytes)
    return h.value, d.value


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", default="dev", choices=("dev", "psi_host", "all_host", "arrays_host"))
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--calls", type=int, default=500)
    ap.add_argument("--n-max", type=int, default=511)
    a = ap.parse_args()
    B = a.batch
    phys = cfg.DEFAULTS[cfg.IHO].with_(n_max=a.n_max, time_steps=1440, gamma=2 * pi)
    st = Stepper(phys, batch=B, device=0, seed=1)
    N = st.N
    dev = torch.device("cuda", 0)
    psi_d = torch.zeros((B, N), dtype=torch.complex128, device=dev)
    psi_d[:, 0] = 1
    act_d = torch.full((B,), phys.n_actions // 2, dtype=torch.int32, device=dev)
    stp_d = torch.ones((B,), dtype=torch.int32, device=dev)
    noise = torch.randn((1, B, 2), dtype=torch.float64, device=dev)
    q = torch.empty((1, B), dtype=torch.float64, device=dev)
    xm = torch.empty((1, B), dtype=torch.float64, device=dev)
    fs = torch.empty((B,), dtype=torch.int32, device=dev)
    psi_p, act_p, stp_p = psi_d.data_ptr(), act_d.data_ptr(), stp_d.data_ptr()
    if a.variant in ("psi_host", "all_host"):
        hp, psi_p = mapped(B * N * 16)
        src = psi_d.cpu().numpy()
        ctypes.memmove(hp, src.ctypes.data, src.nbytes)
    if a.variant in ("arrays_host", "all_host"):
        ha, act_p = mapped(B * 4)
        hs, stp_p = mapped(B * 4)
        np.ctypeslib.as_array((ctypes.c_int32 * B).from_address(ha))[:] = phys.n_actions // 2
        np.ctypeslib.as_array((ctypes.c_int32 * B).from_address(hs))[:] = 1
    torch.cuda.synchronize()
    lib = L.lib()

    def call():
        st._bind_stream()
        L.check(lib.qc_step(st._h, psi_p, act_p, phys.n_actions // 2, 1, stp_p, noise.data_ptr(), q.data_ptr(),
                            xm.data_ptr(), fs.data_ptr(), None, None), st._h)
        L.check(lib.qc_sync(st._h), st._h)
    for _ in range(50):
        call()
    ts = []
    for _ in range(a.calls):
        t0 = time.perf_counter()
        call()
        ts.append(time.perf_counter() - t0)
    print(json.dumps({"variant": a.variant, "batch": B, "us_per_call_median": float(np.median(ts) * 1e6),
                      "us_per_call_p10": float(np.percentile(ts, 10) * 1e6)}))


if __name__ == "__main__":
    main()
