import os
import subprocess
import sys
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _selects_gpu(config) -> bool:
    m = (config.getoption("markexpr", "") or "").replace(" ", "")
    return "gpu" in m and "notgpu" not in m


def _start_rccl_child(config):
    """tests/test_gpu_rccl.py: the bench.py runs of tests/bench_children.py (RCCL at world 1, the two-rank
    launcher rehearsal on one device, the one-rank whole batch). Started here, before collection imports any
    module that initialises the GPU in this process, so every child is a fresh program started by a process
    that never touched the GPU."""
    outdir = tempfile.mkdtemp(prefix="qcart_bench_children_")
    log = open(os.path.join(outdir, "runner.log"), "w")
    proc = subprocess.Popen([sys.executable, "-m", "tests.bench_children", outdir], cwd=ROOT, stdout=log,
                            stderr=subprocess.STDOUT)
    config._qcart_rccl = (proc, outdir)


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
        h[0].terminate()          # the runner kills its running bench group (tests/bench_children.py)
        try:
            h[0].wait(timeout=30)
        except subprocess.TimeoutExpired:
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
