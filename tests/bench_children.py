"""bench.py runs for the GPU suite, started by tests/conftest.py before the pytest process touches the GPU and
run one after another (python -m tests.bench_children <outdir>); tests/test_gpu_rccl.py reads their logs.

  rccl    bench.py's rank body under a launcher's environment at WORLD_SIZE = 1: an RCCL communicator of one rank
  share2  `bench.py --gpus 2` through bench.py's own launcher with QCART_BENCH_SHARE_DEVICE=1: both ranks on
          device 0, gloo carrying the collectives (the N-rank path rehearsed on a one-GPU lease)
  whole1  a plain one-rank run of the two ranks' envs together, for the shard-digest comparison
  trun2   the driver's own launch, `python -m torch.distributed.run --nproc-per-node 2 ... bench.py --gpus 2`, with
          QCART_BENCH_SHARE_DEVICE=1 (both ranks on device 0, gloo)

Each run is a process group of its own, bounded at 300 s (then killed whole, rc 124); after the first failure
nothing more is started; SIGTERM kills the running group and ends the runner. Writes <name>.log (stdout +
stderr) and <name>.rc."""
import os
import signal
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BATCH = 512          # envs per rank
COMMON = ["--steps", "3", "--warmup", "1", "--no-cpu-baseline"]


def runs():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    base = {k: v for k, v in os.environ.items()
            if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    base["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    bench = os.path.join(ROOT, "bench.py")
    yield "rccl", dict(base, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", LOCAL_WORLD_SIZE="1",
                       MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port)), \
        [bench, "--gpus", "1", "--batch", str(BATCH)] + COMMON
    yield "share2", dict(base, QCART_BENCH_SHARE_DEVICE="1"), \
        [bench, "--gpus", "2", "--batch", str(BATCH), "--digest-envs", str(BATCH), "--launch-timeout", "240"] + COMMON
    yield "whole1", base, [bench, "--gpus", "1", "--batch", str(2 * BATCH), "--digest-envs", str(BATCH)] + COMMON
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port2 = sk.getsockname()[1]
    yield "trun2", dict(base, QCART_BENCH_SHARE_DEVICE="1"), \
        ["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
         "--master-port", str(port2), bench, "--gpus", "2", "--batch", str(BATCH), "--digest-envs", str(BATCH)] + COMMON


LIMIT_S = 300
_current = []


def _kill_current(*_):
    for p in _current:
        try:
            os.killpg(p.pid, signal.SIGKILL)
        except ProcessLookupError:
            pass
    sys.exit(143)


def main(outdir: str) -> int:
    signal.signal(signal.SIGTERM, _kill_current)
    for name, env, argv in runs():
        with open(os.path.join(outdir, name + ".log"), "w") as log:
            p = subprocess.Popen([sys.executable, "-u"] + argv, cwd=ROOT, env=env, stdout=log,
                                 stderr=subprocess.STDOUT, start_new_session=True)
            _current[:] = [p]
            try:
                rc = p.wait(timeout=LIMIT_S)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()
                rc = 124
            _current.clear()
        with open(os.path.join(outdir, name + ".rc"), "w") as f:
            f.write(str(rc))
        if rc != 0:
            return rc
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
