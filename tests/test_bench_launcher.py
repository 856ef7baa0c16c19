"""bench.py's own launcher: `--gpus N` without an external torchrun starts N rank processes (before any
GPU call) that join one process group; --dry-run checks it with gloo on the CPU."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, env=None):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=e, capture_output=True,
                          text=True, timeout=180)


def test_launcher_starts_world_of_two():
    out = _run("--gpus", "2", "--dry-run")
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [json.loads(x) for x in out.stdout.splitlines() if x.startswith("{")]
    assert lines == [{"dry_run": True, "n_gpus": 2, "world_size_seen": 2}]


def test_gpus_must_match_external_world_size():
    out = _run("--gpus", "4", "--dry-run", env={"WORLD_SIZE": "2", "RANK": "0"})
    assert out.returncode != 0 and "WORLD_SIZE=2" in out.stderr


def test_failed_rank_stops_the_job_fast():
    """A rank that dies at start (QCART_BENCH_FAIL_RANK: exit 3 before joining the group) must not leave its
    sibling blocked in the rendezvous: the launcher kills it and returns the failed rank's code with its
    stderr tail, within seconds."""
    import time
    t0 = time.monotonic()
    out = _run("--gpus", "2", "--dry-run", env={"QCART_BENCH_FAIL_RANK": "1"})
    dt = time.monotonic() - t0
    assert out.returncode == 3, (out.returncode, out.stderr[-2000:])
    assert dt < 30, dt
    assert "rank 1 of 2 exited with code 3" in out.stderr
    assert "QCART_BENCH_FAIL_RANK" in out.stderr.split("Its stderr tail:")[-1]
    assert not [x for x in out.stdout.splitlines() if x.startswith("{")]


def test_failed_rank_zero_stops_the_job_fast():
    import time
    t0 = time.monotonic()
    out = _run("--gpus", "3", "--dry-run", env={"QCART_BENCH_FAIL_RANK": "0"})
    assert out.returncode == 3 and time.monotonic() - t0 < 30, out.stderr[-2000:]
    assert "rank 0 of 3 exited with code 3" in out.stderr


def test_launch_deadline_kills_hung_ranks():
    """--launch-timeout bounds the whole job: a rank that hangs before joining (QCART_BENCH_HANG_RANK) leaves
    rank 0 waiting in the rendezvous; at the deadline both are killed and the launcher returns 124."""
    import time
    t0 = time.monotonic()
    out = _run("--gpus", "2", "--dry-run", "--launch-timeout", "5",
               env={"QCART_BENCH_HANG_RANK": "1", "QCART_DIST_TIMEOUT_S": "120"})
    assert out.returncode == 124 and time.monotonic() - t0 < 30, out.stderr[-2000:]
    assert "all ranks killed" in out.stderr


def test_torchrun_launch_dry_run():
    """The driver's launch (python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 ...
    bench.py --gpus 2): the ranks take RANK / WORLD_SIZE from torchrun and join one group."""
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                          "--gpus", "2", "--dry-run"], env=e, capture_output=True, text=True, timeout=180)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [json.loads(x) for x in out.stdout.splitlines() if x.startswith("{")]
    assert lines == [{"dry_run": True, "n_gpus": 2, "world_size_seen": 2}]
