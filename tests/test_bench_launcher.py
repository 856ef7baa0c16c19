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
