"""The step server's shared-memory protocol on the CPU (no GPU): libqcart_client.so against a mock server
thread that plays qcart_server.cpp's side of csrc/qcart_shm.h (slot claim, request / done sequence numbers,
the tick futex), plus the layout mirror checked against the C header with gcc."""
import ctypes
import mmap
import os
import shutil
import subprocess
import threading
import time

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "deepreinforcementlearningcontrolofquantumcartpoles_amd")
CLIENT = os.path.join(PKG, "libqcart_client.so")
SHM_H = os.path.join(PKG, "csrc", "qcart_shm.h")

pytestmark = pytest.mark.skipif(not os.path.exists(CLIENT), reason="libqcart_client.so not built")

u32, i32, u64, d = ctypes.c_uint32, ctypes.c_int32, ctypes.c_uint64, ctypes.c_double


class Header(ctypes.Structure):
    _fields_ = [("magic", u32), ("version", u32), ("max_clients", i32), ("N", i32), ("n_obs", i32), ("family", i32),
                ("alive", u32), ("tick", u32), ("kick", u32), ("server_sleeping", u32), ("n_clients", u32),
                ("server_pid", i32), ("slot_off", u64), ("psi_off", u64), ("obs_off", u64), ("total_bytes", u64),
                ("n_max", i32), ("moment_order", i32), ("omega", d), ("x_max", d), ("grid_size", d), ("lambda_", d),
                ("mass", d), ("f_max", d), ("n_actions", i32), ("pad1", i32), ("ticks", u64), ("calls", u64),
                ("pid_ns", u64), ("r_on", u32), ("r_gen", u32), ("r_dt", d), ("r_gamma", d), ("r_pad1", u64 * 8),
                ("r_quit", u32), ("r_beat", u32), ("r_pad2", u64 * 7)]


class Slot(ctypes.Structure):
    _fields_ = [("owner", u32), ("pid", i32), ("req", u32), ("done", u32), ("waiting", u32), ("op", i32), ("n", i32),
                ("seed", u32), ("dt", d), ("force", d), ("gamma", d), ("status", i32), ("fail", i32), ("q", d),
                ("xmean", d), ("value", d), ("err", ctypes.c_char * 96), ("rreq", u32), ("rdone", u32), ("repoch", u32),
                ("rstatus", i32), ("rcount", u32), ("pad", ctypes.c_uint8 * 12)]


OP_STEP, OP_SET_SEED, OP_X, OP_MOM, OP_FOCK, OP_HDOT = 1, 2, 3, 4, 5, 6
MAX_OBS = 64
VERSION = 3
EBOUNCE = -101


def rq_fields(w):
    """The resident request word (qcart_shm.h QCS_RQ): seq, op, action, generation, epoch, keep."""
    return w & 3, (w >> 2) & 3, (w >> 4) & 63, (w >> 10) & 63, (w >> 16) & 0x7fff, w >> 31


def test_layout_mirror_matches_the_c_header(tmp_path):
    if shutil.which("gcc") is None:
        pytest.skip("no gcc")
    src = tmp_path / "lay.c"
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{SHM_H}"', "int main(void){"]
    for S, c in ((Header, "qcs_header"), (Slot, "qcs_slot")):
        for f, _ in S._fields_:
            lines.append(f'printf("%zu\\n", offsetof({c}, {f}));')
        lines.append(f'printf("%zu\\n", sizeof({c}));')
    lines.append("return 0;}")
    src.write_text("\n".join(lines))
    exe = tmp_path / "lay"
    subprocess.run(["gcc", str(src), "-o", str(exe)], check=True)
    got = [int(v) for v in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]
    want = []
    for S in (Header, Slot):
        want += [getattr(S, f).offset for f, _ in S._fields_] + [ctypes.sizeof(S)]
    assert got == want
    hdr_off = {f: getattr(Header, f).offset for f, _ in Header._fields_}
    assert hdr_off["r_quit"] % 64 == 0 and hdr_off["r_on"] < 256   # the GPU-polled words on a line of their own


class MockServer:
    """qcart_server.cpp's side of the protocol in Python: STEP negates the state and reports q = 1.5 n,
    x_mean = force, Fail = n == 10; SET_SEED stores the seed in `value`; X_EXPECT returns the sum of Re(psi);
    MOMENTS fills the obs row with 0, 1, 2, ...; HDOT doubles the row. serve_ops: the ops it answers (others stay
    pending forever: a server that hangs on them). resident: it also plays the resident kernel (r_on, the request
    word rreq / rdone: a step multiplies the row by 3, q = 100 + action, x_mean = force, Fail 0; x_expectation returns
    minus the sum of Re(psi); the observation row 100, 101, ...), bouncing action `bounce` and steps of another
    dynamics generation than r_gen to the ticks."""

    def __init__(self, name, P=3, N=8, n_obs=5, serve_ops=None, resident=False, bounce=-1, grid_kernel=False):
        self.name, self.P, self.N, self.n_obs = name, P, N, n_obs
        self.serve_ops = serve_ops
        rnd = lambda v: (v + 4095) // 4096 * 4096   # noqa: E731
        self.slot_off = rnd(ctypes.sizeof(Header))
        self.psi_off = rnd(self.slot_off + ctypes.sizeof(Slot) * P)
        self.obs_off = rnd(self.psi_off + 16 * N * P)
        self.total = rnd(self.obs_off + 8 * MAX_OBS * P)
        path = "/dev/shm" + name
        with open(path, "wb") as f:
            f.truncate(self.total)
        self.fd = os.open(path, os.O_RDWR)
        self.mm = mmap.mmap(self.fd, self.total)
        self.hdr = Header.from_buffer(self.mm, 0)
        self.slots = (Slot * P).from_buffer(self.mm, self.slot_off)
        self.psi = np.frombuffer(self.mm, np.complex128, N * P, self.psi_off).reshape(P, N)
        self.obs = np.frombuffer(self.mm, np.float64, MAX_OBS * P, self.obs_off).reshape(P, MAX_OBS)
        h = self.hdr
        h.magic, h.version, h.max_clients, h.N, h.n_obs, h.family = 0x56534351, VERSION, P, N, n_obs, 1
        h.f_max, h.n_actions = 8.0, 21
        self.bounce = bounce
        self.grid_kernel = grid_kernel   # a grid family's resident kernel: every non-step op bounces (the reset too)
        self.kernel_gen = None   # the "kernel's" generation (None: the header's)
        if resident:
            h.r_on, h.r_dt, h.r_gamma = 1, 1 / 1440, 6.28
        h.server_pid, h.pid_ns = os.getpid(), os.stat("/proc/self/ns/pid").st_ino
        h.slot_off, h.psi_off, h.obs_off, h.total_bytes = self.slot_off, self.psi_off, self.obs_off, self.total
        h.n_max, h.omega = N - 1, 3.14159
        h.alive = 1
        self.served = [0] * P
        self.rserved = [0] * P
        self.stop = False
        self.libc = ctypes.CDLL(None, use_errno=True)
        self.t = threading.Thread(target=self.loop, daemon=True)
        self.t.start()

    def loop(self):
        while not self.stop:
            any_ = False
            for e in range(self.P):
                s = self.slots[e]
                if self.hdr.r_on and s.owner and s.rreq != self.rserved[e]:
                    _, op, act, gen, _, _ = rq_fields(s.rreq)
                    kgen = self.hdr.r_gen if self.kernel_gen is None else self.kernel_gen
                    if op == 3:
                        s.rstatus = EBOUNCE if self.grid_kernel else 0
                    elif op != 0 and self.grid_kernel:
                        s.rstatus = EBOUNCE
                    elif op == 1:
                        s.value, s.rstatus = -float(self.psi[e].real.sum()), 0
                    elif op == 2:
                        self.obs[e, :self.n_obs] = 100 + np.arange(self.n_obs)
                        s.rstatus = 0
                    elif act == self.bounce or gen != (kgen & 63):
                        s.rstatus = EBOUNCE
                    else:
                        self.psi[e] *= 3
                        s.q, s.xmean, s.fail, s.rstatus = 100.0 + act, s.force, 0, 0
                    s.rcount += 1
                    self.rserved[e] = s.rreq
                    s.rdone = s.rreq
                    any_ = True
                if not s.owner or s.req == self.served[e]:
                    continue
                if self.serve_ops is not None and s.op not in self.serve_ops:
                    continue
                any_ = True
                if s.op == OP_STEP:
                    self.psi[e] *= -1
                    s.q, s.xmean, s.fail = 1.5 * s.n, s.force, int(s.n == 10)
                elif s.op == OP_SET_SEED:
                    s.value = float(s.seed)
                elif s.op == OP_X:
                    s.value = float(self.psi[e].real.sum())
                elif s.op == OP_HDOT:
                    self.psi[e] *= 2
                else:
                    self.obs[e, :self.n_obs] = np.arange(self.n_obs)
                s.status = 0
                self.served[e] = s.req
                s.done = s.req
            if any_:
                self.hdr.tick += 1
                addr = ctypes.addressof(self.hdr) + Header.tick.offset
                self.libc.syscall(202, ctypes.c_void_p(addr), 1, 1 << 30, None, None, 0)   # FUTEX_WAKE
            else:
                time.sleep(0.0002)

    def close(self):
        self.stop = True
        self.t.join()
        self.hdr.alive = 0
        del self.hdr, self.slots, self.psi, self.obs
        self.mm.close()
        os.close(self.fd)
        os.unlink("/dev/shm" + self.name)


def _client_module():
    from deepreinforcementlearningcontrolofquantumcartpoles_amd import simulation as S
    return S


def test_client_without_server_fails_loudly():
    L = _client_module()._client_lib()
    c = ctypes.c_void_p()
    rc = L.qcc_open(b"/qcart_no_such_server", ctypes.byref(c))
    assert rc == -7 and not c.value
    assert b"no step server" in L.qcc_last_error(None)


def test_client_calls_through_the_protocol():
    S = _client_module()
    from deepreinforcementlearningcontrolofquantumcartpoles_amd import config as cfg
    srv = MockServer(f"/qcart_mock_{os.getpid()}", P=2, N=8)
    try:
        ph = cfg.DEFAULTS[cfg.IHO].with_(n_max=7, omega=3.14159)
        a = S._ServedSimulation(ph, srv.name)
        b = S._ServedSimulation(ph, srv.name)
        with pytest.raises(RuntimeError, match="slots are taken"):
            S._ServedSimulation(ph, srv.name)
        assert srv.hdr.n_clients == 2
        state = (np.arange(8) + 1j).astype(np.complex128)
        q, xm, fail = a.step(state, 1 / 1440, 0.8, 6.28)
        assert (q, xm, fail) == (1.5, 0.8, 0) and np.array_equal(state, -(np.arange(8) + 1j))
        q, xm, fail = b.simulate_10_steps(state, 1 / 1440, -1.6, 6.28)
        assert (q, xm, fail) == (15.0, -1.6, 1) and np.array_equal(state, np.arange(8) + 1j)
        assert a.Hamiltonian_dot_psi(state) == 0.0 and np.array_equal(state, 2 * (np.arange(8) + 1j))
        state /= 2
        with pytest.raises(NotImplementedError):
            a.solve_ab(state)
        a.set_seed(2 ** 32 + 77)                        # the int's low 32 bits, as the reference's MKL_UINT
        assert srv.slots[0].value == 77.0
        assert a.x_expectation(state) == float(np.arange(8).sum())
        with pytest.raises(ValueError, match="required size 8"):
            a.step(np.zeros(9, np.complex128), 1 / 1440, 0.0, 6.28)
        # concurrent callers: every call answered with its own slot's data
        errs = []

        def run(m, sign):
            st = np.full(8, sign, np.complex128)
            for _ in range(200):
                m.step(st, 1 / 1440, 0.0, 6.28)
            if not np.array_equal(st, np.full(8, sign)):
                errs.append(sign)
        ts = [threading.Thread(target=run, args=(m, s)) for m, s in ((a, 1.0), (b, -2.0))]
        [t.start() for t in ts]
        [t.join() for t in ts]
        assert not errs
        a.close()
        assert srv.slots[0].owner == 0 and srv.hdr.n_clients == 1
        c = S._ServedSimulation(ph, srv.name)   # the freed slot is claimed again
        b.close()
        c.close()
        # a mismatched module (the drivers' check_settings handshake) is refused
        with pytest.raises(RuntimeError, match="serves family"):
            S._ServedSimulation(ph.with_(n_max=15), srv.name)
    finally:
        srv.close()


def test_client_takes_the_resident_path():
    """A server with a resident kernel (r_on): step(state, dt, force, gamma) on the action grid at r_dt / r_gamma goes
    through rreq / rdone; an off-grid force, another dt or gamma, simulate_10_steps and a bounced request (the
    kernel's QCS_EBOUNCE) go through the ticks; qcc_close waits for neither path."""
    S = _client_module()
    from deepreinforcementlearningcontrolofquantumcartpoles_amd import config as cfg
    srv = MockServer(f"/qcart_mockr_{os.getpid()}", P=2, N=8, resident=True, bounce=10)
    try:
        ph = cfg.DEFAULTS[cfg.IHO].with_(n_max=7, omega=3.14159)
        a = S._ServedSimulation(ph, srv.name)
        base = (np.arange(8) + 1j).astype(np.complex128)
        st = base.copy()
        q, xm, fail = a.step(st, 1 / 1440, 0.8, 6.28)            # grid action 11 (spacing 0.8): resident
        assert (q, xm, fail) == (111.0, 0.8, 0) and np.array_equal(st, 3 * base)
        assert rq_fields(srv.slots[0].rreq)[5] == 0              # the first call: the row read from the slot
        a.step(st, 1 / 1440, 0.8, 6.28)                          # the state as returned: `keep`
        assert rq_fields(srv.slots[0].rreq)[5] == 1 and np.array_equal(st, 9 * base)
        st[0] += 1                                               # changed by the driver: read again
        a.step(st, 1 / 1440, 0.8, 6.28)
        assert rq_fields(srv.slots[0].rreq)[5] == 0
        st = base.copy()
        q, xm, fail = a.step(st, 1 / 1440, -8.0, 6.28)           # action 0
        assert q == 100.0 and np.array_equal(st, 3 * base)
        st = base.copy()
        q, xm, fail = a.step(st, 1 / 1440, 0.0, 6.28)            # action 10: bounced -> the tick path
        assert (q, xm, fail) == (1.5, 0.0, 0) and np.array_equal(st, -base)
        for args in ((1 / 1440, 0.7, 6.28), (1 / 2880, 0.8, 6.28), (1 / 1440, 0.8, 3.14)):   # off grid, dt, gamma
            st = base.copy()
            q, xm, fail = a.step(st, *args)
            assert q == 1.5 and np.array_equal(st, -base), args
        st = base.copy()
        q, xm, fail = a.simulate_10_steps(st, 1 / 1440, 0.8, 6.28)
        assert (q, fail) == (15.0, 1) and np.array_equal(st, -base)
        # the resident requests so far: the open's reset and 5 steps; every call that took stream words through the
        # ticks (and the open's set_seed) moved the epoch: 1 + the bounce + 3 + simulate_10_steps = 6
        s0 = srv.slots[0]
        assert s0.rreq == s0.rdone and s0.repoch == 6 and s0.rcount == 6
        st = base.copy()
        a.step(st, 1 / 1440, 1.6, 6.28)
        _, op, act, gen, ep, keep = rq_fields(s0.rreq)
        assert (op, act, gen, ep, keep) == (0, 12, 0, 6, 0)
        # x_expectation and the observation vector on the resident path too (op 1, 2), the stream untouched
        assert a.x_expectation(st) == -float(st.real.sum()) and rq_fields(s0.rreq)[1] == 1 and s0.repoch == 6
        data = np.zeros(5)
        a.get_moments(st, data)
        assert np.array_equal(data, 100 + np.arange(5.0)) and rq_fields(s0.rreq)[1] == 2
        # 2^15 tick-path draws since the last resident step would alias in the word's 15 epoch bits: the client moves
        # the epoch on once more
        last = rq_fields(s0.rreq)[4]
        s0.repoch += 0x8000
        st = base.copy()
        a.step(st, 1 / 1440, 1.6, 6.28)
        assert rq_fields(s0.rreq)[4] == (last + 1) & 0x7fff and s0.repoch == 6 + 0x8000 + 1
        srv.kernel_gen = 5                                # a relaunch after a dynamics change: generation 0 bounces
        st = base.copy()
        assert a.step(st, 1 / 1440, 1.6, 6.28)[0] == 1.5 and rq_fields(s0.rreq)[3] == 0
        srv.hdr.r_gen = 5                                 # ... and the header's: the client's requests carry it
        st = base.copy()
        assert a.step(st, 1 / 1440, 1.6, 6.28)[0] == 112.0 and rq_fields(s0.rreq)[3] == 5
        del s0
        t0 = time.monotonic()
        a.close()
        assert time.monotonic() - t0 < 1.0 and srv.hdr.n_clients == 0
    finally:
        srv.close()


def test_client_opens_on_a_grid_resident_kernel():
    """A grid family's resident kernel answers the reset a new owner sends at open with a bounce (every non-step op
    bounces there): the module still opens, and its steps take the resident path."""
    S = _client_module()
    from deepreinforcementlearningcontrolofquantumcartpoles_amd import config as cfg
    srv = MockServer(f"/qcart_mockg_{os.getpid()}", P=1, N=8, resident=True, grid_kernel=True)
    try:
        a = S._ServedSimulation(cfg.DEFAULTS[cfg.IHO].with_(n_max=7, omega=3.14159), srv.name)
        s0 = srv.slots[0]
        assert rq_fields(s0.rreq)[1] == 3 and s0.rstatus == EBOUNCE and s0.rcount == 1
        base = (np.arange(8) + 1j).astype(np.complex128)
        st = base.copy()
        q, xm, fail = a.step(st, 1 / 1440, 0.8, 6.28)
        assert q == 111.0 and np.array_equal(st, 3 * base) and s0.rcount == 2
        del s0
        a.close()
    finally:
        srv.close()


_DYING = """
import sys, time
sys.path.insert(0, {root!r})
from tests.test_server_protocol import MockServer, OP_SET_SEED
srv = MockServer({name!r}, P=2, N=8, serve_ops={{OP_SET_SEED}})   # answers set_seed (qcc_open's), never a step
print("ready", flush=True)
time.sleep(600)
"""


def test_client_detects_a_killed_server():
    """A server killed without clearing `alive` (SIGKILL, a GPU-fault abort): a client waiting on it fails within a
    second (the 20 ms liveness check reads the server's pid), qcc_close returns, and the object it left behind is
    refused by the next qcc_open."""
    import signal
    import sys
    S = _client_module()
    from deepreinforcementlearningcontrolofquantumcartpoles_amd import config as cfg
    name = f"/qcart_dying_{os.getpid()}"
    proc = subprocess.Popen([sys.executable, "-c", _DYING.format(root=ROOT, name=name)], cwd=ROOT,
                            stdout=subprocess.PIPE, text=True)
    try:
        assert proc.stdout.readline().strip() == "ready"
        ph = cfg.DEFAULTS[cfg.IHO].with_(n_max=7, omega=3.14159)
        a = S._ServedSimulation(ph, name)
        out = {}

        def call():
            t0 = time.monotonic()
            try:
                a.step(np.zeros(8, np.complex128), 1 / 1440, 0.0, 6.28)
            except RuntimeError as e:
                out["err"] = str(e)
            out["dt"] = time.monotonic() - t0
        th = threading.Thread(target=call)
        th.start()
        time.sleep(0.3)
        assert th.is_alive()                      # the step is pending: the server never answers it
        t_kill = time.monotonic()
        proc.send_signal(signal.SIGKILL)
        proc.wait()
        th.join(timeout=10)
        assert not th.is_alive()
        assert "exited" in out["err"] and time.monotonic() - t_kill < 2.0, out
        t0 = time.monotonic()
        a.close()                                 # the pending request does not hold the close
        assert time.monotonic() - t0 < 1.0
        with pytest.raises(RuntimeError, match="no live step server"):
            S._ServedSimulation(ph, name)
    finally:
        if proc.poll() is None:
            proc.kill()
            proc.wait()
        if os.path.exists("/dev/shm" + name):
            os.unlink("/dev/shm" + name)
