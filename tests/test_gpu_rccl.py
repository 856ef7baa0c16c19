"""bench.py's multi-rank path on a GPU (SURVEY §4 item 4's "fake cluster"; reference model
IHO/main_parallel.py:345-359, one process per worker).

tests/conftest.py starts tests/bench_children.py before this process touches the GPU; it runs, one after
another:
  rccl    bench.py's rank body under a launcher's environment at WORLD_SIZE = 1: the rank joins a
          torch.distributed "nccl" (= RCCL) group, times its shard between barriers, max-reduces the timing with
          all_reduce and gathers every env's episode statistics with distributed.gather_episode_stats on device
          tensors;
  share2  `bench.py --gpus 2` through bench.py's own launcher with QCART_BENCH_SHARE_DEVICE=1: two ranks on
          device 0, gloo carrying the same collectives — the path the driver's 8-GPU run takes, on one GPU;
  whole1  one plain rank stepping both ranks' envs (2B) — rank r's shard must equal envs [rB, (r+1)B) of it bit
          for bit (inputs, psi0 and noise are keyed by the global env id);
  trun2   the driver's launch (torch.distributed.run, 2 processes) on one device.
These tests read the runs' JSON lines."""
import json
import os

import pytest

from tests.bench_children import BATCH

pytestmark = pytest.mark.gpu


def _wait(request):
    h = getattr(request.config, "_qcart_rccl", None)
    if h is None:
        pytest.skip("the bench children are started only by a `-m gpu` session on a GPU box")
    proc, outdir = h
    proc.wait(timeout=960)
    return outdir


def _result(outdir, name):
    log = os.path.join(outdir, name + ".log")
    rcf = os.path.join(outdir, name + ".rc")
    runner = open(os.path.join(outdir, "runner.log")).read()
    assert os.path.exists(rcf), f"{name} did not run (an earlier run failed?)\n" + runner[-2000:]
    text = open(log).read()
    rc = int(open(rcf).read())
    assert rc == 0, f"{name}: rc {rc}\n" + text[-3000:]
    lines = [ln for ln in text.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, text[-3000:]            # rank 0 alone prints, once
    return json.loads(lines[0])


@pytest.mark.timeout(1000)
def test_bench_rank_body_runs_rccl_at_world_size_1(request):
    res = _result(_wait(request), "rccl")
    assert res["n_gpus"] == 1 and res["config"]["world_size_seen"] == 1
    r = res["config"]["rccl"]
    assert r is not None and r["backend"] == "nccl" and r["world_size"] == 1 and not r["share_device"]
    assert r["device"].startswith("cuda")
    assert r["gathered_envs"] == BATCH              # every env's statistics came back through the gather
    assert 0 <= r["gathered_survivors"] <= BATCH
    assert res["value"] > 0 and res["roofline"]["kernel_launches"] == 3


@pytest.mark.timeout(1000)
def test_two_rank_launch_on_one_device(request):
    """bench.py --gpus 2 with its own launcher: world 2 seen, the global batch and the gathered envs are 2B, the
    value counts both ranks' env-steps over the max-over-ranks time."""
    res = _result(_wait(request), "share2")
    assert res["n_gpus"] == 2 and res["config"]["world_size_seen"] == 2
    assert res["config"]["global_batch"] == 2 * BATCH
    r = res["config"]["rccl"]
    assert r["world_size"] == 2 and r["backend"] == "gloo" and r["share_device"]
    assert r["gathered_envs"] == 2 * BATCH and 0 <= r["gathered_survivors"] <= 2 * BATCH
    n_sub = res["config"]["physics_steps_per_step"]
    units = 2 * BATCH * n_sub * res["steps"]
    assert abs(res["value"] * res["ms_per_step"] * res["steps"] / 1e3 - units) < 1e-6 * units
    assert res["roofline"]["kernel_launches"] == 3


@pytest.mark.timeout(1000)
def test_rank_shards_equal_the_one_rank_run_bitwise(request):
    outdir = _wait(request)
    two = _result(outdir, "share2")["psi_digests"]
    one = _result(outdir, "whole1")["psi_digests"]
    assert len(two) == 2 and len(one) == 2
    assert two == one                               # rank r's final psi == envs [rB, (r+1)B) of the 2B run
    assert two[0] != two[1]


@pytest.mark.timeout(1000)
def test_torchrun_launch_on_one_device(request):
    """The driver's own N-rank launch (python -m torch.distributed.run --nproc-per-node 2 ... bench.py --gpus 2): world
    2, one JSON line from rank 0, the same shard digests as bench.py's own launcher."""
    outdir = _wait(request)
    res = _result(outdir, "trun2")
    assert res["n_gpus"] == 2 and res["config"]["world_size_seen"] == 2
    assert res["config"]["rccl"]["gathered_envs"] == 2 * BATCH
    assert res["psi_digests"] == _result(outdir, "whole1")["psi_digests"]
