"""The RCCL code path on a GPU at world size 1 (SURVEY §4 item 4's one-rank "fake cluster"; reference
model IHO/main_parallel.py:345-359, one process per worker).

tests/conftest.py starts, before this process touches the GPU, `bench.py --gpus 1` with a launcher's
environment (WORLD_SIZE=1, RANK=0, MASTER_ADDR=127.0.0.1): the rank joins a torch.distributed "nccl"
(= RCCL) group, times its shard between barriers, max-reduces the timing with all_reduce and gathers
every env's episode statistics with distributed.gather_episode_stats on device tensors. This test reads
the rank's JSON line."""
import json

import pytest

pytestmark = pytest.mark.gpu


def test_bench_rank_body_runs_rccl_at_world_size_1(request):
    h = getattr(request.config, "_qcart_rccl", None)
    if h is None:
        pytest.skip("the RCCL child is started only by a `-m gpu` session on a GPU box")
    from tests.conftest import RCCL_BATCH
    proc, log = h
    rc = proc.wait(timeout=320)
    text = open(log).read()
    assert rc == 0, text[-3000:]
    line = [ln for ln in text.splitlines() if ln.startswith("{")][-1]
    res = json.loads(line)
    assert res["n_gpus"] == 1 and res["config"]["world_size_seen"] == 1
    r = res["config"]["rccl"]
    assert r is not None and r["backend"] == "nccl" and r["world_size"] == 1
    assert r["device"].startswith("cuda")
    assert r["gathered_envs"] == RCCL_BATCH            # every env's statistics came back through the gather
    assert 0 <= r["gathered_survivors"] <= RCCL_BATCH
    assert res["value"] > 0 and res["roofline"]["kernel_launches"] == 3
