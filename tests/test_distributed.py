"""Multi-process (gloo, world_size 2, CPU) coverage of the N>1 path: env sharding, the episode-stat
gather that RCCL carries on the GPU node, and the invariance of trajectories to the sharding
(noise keyed by global env id; checked with the CPU oracle as the checker)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from deepreinforcementlearningcontrolofquantumcartpoles_amd import distributed as D


def test_shard_partitions_exactly():
    for gb in (1, 7, 64, 65536, 65537):
        for w in (1, 2, 3, 8):
            parts = [D.shard(gb, w, r) for r in range(w)]
            assert sum(c for _, c in parts) == gb
            off = 0
            for o, c in parts:
                assert o == off
                off += c
    with pytest.raises(ValueError):
        D.shard(8, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # ragged per-rank episode lists
        n = 3 + 2 * rank
        ret = torch.arange(n, dtype=torch.float64) + 100 * rank
        ln = torch.full((n,), 10.0 * (rank + 1))
        R, L = D.gather_episode_stats(ret, ln)
        m = D.max_over_ranks(float(rank) + 0.5)
        # sharded oracle trajectories (the checker) keyed by global env id
        from oracle import oracle as O
        from deepreinforcementlearningcontrolofquantumcartpoles_amd import config as cfg
        ph = cfg.DEFAULTS[cfg.IHO].with_(n_max=63)
        s = O.OracleSystem(ph.family, n_max=ph.n_max)
        off, cnt = D.shard(6, world, rank)
        psi = np.stack([s.fock_random_state(1, off + e, 16) for e in range(cnt)])
        acts = (np.arange(off, off + cnt) % 21).astype(np.int32)
        s.run_batch(psi, acts, ph.f_max, 30, ph.dt, ph.gamma, seed=5, env_offset=off, n_threads=1)
        q.put((rank, R.tolist(), L.tolist(), m, off, psi))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_gather_and_shard_invariance(oracle_mod):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r = q.get(timeout=180)
        res[r[0]] = r
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    exp_R = [0.0, 1.0, 2.0] + [100.0 + i for i in range(5)]
    exp_L = [10.0] * 3 + [20.0] * 5
    for r in (0, 1):
        assert res[r][1] == exp_R and res[r][2] == exp_L and res[r][3] == 1.5
    # single-process run of all 6 envs == concatenation of the two shards (bitwise)
    from deepreinforcementlearningcontrolofquantumcartpoles_amd import config as cfg
    ph = cfg.DEFAULTS[cfg.IHO].with_(n_max=63)
    s = oracle_mod.OracleSystem(ph.family, n_max=ph.n_max)
    psi = np.stack([s.fock_random_state(1, e, 16) for e in range(6)])
    s.run_batch(psi, (np.arange(6) % 21).astype(np.int32), ph.f_max, 30, ph.dt, ph.gamma, seed=5, n_threads=1)
    assert np.array_equal(np.concatenate([res[0][5], res[1][5]]), psi)
