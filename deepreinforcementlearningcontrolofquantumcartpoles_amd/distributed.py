"""Multi-GPU: one process per GPU, each owning a contiguous shard of global env ids.

Envs never interact (the reference already runs them as independent actor processes,
IHO/main_parallel.py:345-359), so the data path has no collective: every rank steps its shard
with its own libqcart handle (env_offset = first global id of the shard keeps the Philox noise,
and therefore the trajectories, identical to a 1-GPU run). RCCL over xGMI (torch.distributed
backend "nccl") is used only to gather episode statistics (returns, lengths) at report time —
a few KB, latency-bound.
"""
from __future__ import annotations

import datetime
import os
from typing import Tuple

import torch
import torch.distributed as dist


def shard(global_batch: int, world: int, rank: int) -> Tuple[int, int]:
    """(env_offset, count) of rank's contiguous shard; the first global_batch % world ranks get one more."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    base, extra = divmod(int(global_batch), int(world))
    count = base + (1 if rank < extra else 0)
    offset = rank * base + min(rank, extra)
    return offset, count


# rendezvous and collective timeout: a rank that never joins (it died in RCCL init, or its GPU is gone) fails the
# others in bounded time instead of leaving them blocked for torch's 10-minute default
INIT_TIMEOUT_S = float(os.environ.get("QCART_DIST_TIMEOUT_S", "120"))


def init_from_env(backend: str | None = None) -> Tuple[int, int, int]:
    """Initialise the default process group from torchrun's env (127.0.0.1 rendezvous) whenever a
    launcher started this process — world 1 included, so a one-GPU run under a launcher still goes through
    RCCL (the fake-cluster case of SURVEY §4 item 4). A launcher sets WORLD_SIZE and the rendezvous address;
    a bare WORLD_SIZE=1 without MASTER_ADDR (a user's shell export) is no launcher: nothing is initialised,
    as without WORLD_SIZE."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    launched = "WORLD_SIZE" in os.environ and (world > 1 or "MASTER_ADDR" in os.environ)
    if launched and not dist.is_initialized():
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local),
                                    timeout=datetime.timedelta(seconds=INIT_TIMEOUT_S))
        else:
            dist.init_process_group(backend, timeout=datetime.timedelta(seconds=INIT_TIMEOUT_S))
    return world, rank, local


def gather_episode_stats(returns: torch.Tensor, lengths: torch.Tensor, group=None):
    """All-gather variable-length per-rank episode (return, length) vectors; every rank gets the
    concatenation in rank order. One small all_gather of counts + one of the padded payloads (also at
    world 1 when a process group exists: the collective path is the one that runs)."""
    if not (dist.is_available() and dist.is_initialized()):
        return returns.to(torch.float64), lengths.to(torch.float64)
    world = dist.get_world_size(group)
    dev = returns.device
    n = torch.tensor([returns.numel()], dtype=torch.int64, device=dev)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n, group=group)
    m = int(max(int(c.item()) for c in counts))
    pay = torch.zeros((max(m, 1), 2), dtype=torch.float64, device=dev)
    pay[: returns.numel(), 0] = returns.to(torch.float64).reshape(-1)
    pay[: lengths.numel(), 1] = lengths.to(torch.float64).reshape(-1)
    outs = [torch.zeros_like(pay) for _ in range(world)]
    dist.all_gather(outs, pay, group=group)
    rows = torch.cat([o[: int(c.item())] for o, c in zip(outs, counts)], 0)
    return rows[:, 0], rows[:, 1]


def max_over_ranks(x: float, device=None, group=None) -> float:
    if not (dist.is_available() and dist.is_initialized()):
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())
