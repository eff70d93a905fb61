"""Env sharding across GPUs (one process per GPU) and the learner gather.

SURVEY.md §8e: envs are independent, so each rank steps a contiguous block of envs with no
collective on the data path; the only exchange is returning batched outputs to a single learner
(rank 0) when the trainer is centralised. Global env indices (env_index_base = rank * n_local)
key every random stream, so a sharded run is env-for-env identical to a single-GPU run of the
same total envs (tests/test_distributed.py checks this on gloo).

The reference has no collective at all (single-GPU learner fed by pufferlib worker processes,
clean_pufferl.py:106-114); this module replaces the worker-process IPC of pool.recv()/send()
(:293, :357) with torch.distributed (RCCL over xGMI on MI355X, gloo on CPU).
"""

from __future__ import annotations

import torch
import torch.distributed as dist


def shard(total_envs: int, world: int, rank: int):
    """Contiguous env block of `rank`: (env_index_base, n_local). Requires an even split."""
    if total_envs % world:
        raise ValueError(f"{total_envs} envs do not split evenly over {world} ranks")
    n = total_envs // world
    return rank * n, n


def gather_to_learner(t: torch.Tensor, dst: int = 0):
    """Gather the rank-local batch `t` ([n_local, ...]) to rank `dst` as [world*n_local, ...].
    Each peer -> root transfer is a point-to-point xGMI link under RCCL (no ring)."""
    world = dist.get_world_size()
    if world == 1:
        return t
    if dist.get_rank() == dst:
        bufs = [torch.empty_like(t) for _ in range(world)]
        dist.gather(t.contiguous(), gather_list=bufs, dst=dst)
        return torch.cat(bufs, 0)
    dist.gather(t.contiguous(), dst=dst)
    return None


def scatter_from_learner(full, like: torch.Tensor, src: int = 0) -> torch.Tensor:
    """Scatter [world*n_local, ...] actions from `src` back to every rank's [n_local, ...]."""
    world = dist.get_world_size()
    if world == 1:
        return full
    out = torch.empty_like(like)
    if dist.get_rank() == src:
        chunks = list(full.contiguous().chunk(world, 0))
        dist.scatter(out, scatter_list=chunks, src=src)
    else:
        dist.scatter(out, src=src)
    return out
