import os
import socket
import subprocess
import sys
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

RCCL_BATCH = 512


def _selects_gpu(config) -> bool:
    m = (config.getoption("markexpr", "") or "").replace(" ", "")
    return "gpu" in m and "notgpu" not in m


def _start_rccl_child(config):
    """tests/test_gpu_rccl.py: bench.py's rank body under a launcher's environment at WORLD_SIZE = 1 (an RCCL
    communicator of one rank). Started here, before collection imports any module that initialises the GPU
    in this process, so the child is a fresh program started by a process that never touched the GPU."""
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    out = tempfile.NamedTemporaryFile(prefix="qcart_rccl_", suffix=".log", delete=False)
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", LOCAL_WORLD_SIZE="1",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = ["timeout", "-k", "10", "300", sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1",
           "--steps", "3", "--warmup", "1", "--batch", str(RCCL_BATCH), "--no-cpu-baseline"]
    proc = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=out, stderr=subprocess.STDOUT)
    config._qcart_rccl = (proc, out.name)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: longer CPU test")
    # only the controlling process of a session (pytest-xdist workers carry `workerinput`: each would start a
    # child of its own)
    # with -n (pytest-xdist) the controller never runs pytest_collection_modifyitems (the workers collect), so
    # the child could not be ordered alone before the GPU tests: no child then (test_gpu_rccl skips on the
    # workers); the GPU suite is run without -n
    dist = config.getoption("dist", "no") if hasattr(config.option, "dist") else "no"
    nproc = getattr(config.option, "numprocesses", None)
    if (_selects_gpu(config) and os.path.exists("/dev/kfd") and not hasattr(config, "workerinput")
            and dist == "no" and not nproc):
        _start_rccl_child(config)


def _stop_rccl_child(config):
    h = getattr(config, "_qcart_rccl", None)
    if h is not None and h[0].poll() is None:
        h[0].kill()
        h[0].wait()
    config._qcart_rccl = None


@pytest.hookimpl(trylast=True)   # after -k / -m deselection
def pytest_collection_modifyitems(session, config, items):
    """The RCCL child runs alone on the GPU: its test (which waits for it) goes first, so every other GPU test
    starts after the child has finished; a session that did not collect the test (a -k subset, another
    path) stops the child before any test runs."""
    if getattr(config, "_qcart_rccl", None) is None:
        return
    first = [it for it in items if "test_gpu_rccl.py" in it.nodeid]
    if not first:
        _stop_rccl_child(config)
        return
    items[:] = first + [it for it in items if "test_gpu_rccl.py" not in it.nodeid]


def pytest_unconfigure(config):
    _stop_rccl_child(config)


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle as O
    O.build()
    return O
