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


def gather_wire_to_learner(wire: torch.Tensor, header_bytes: int, dst: int = 0, recv_bufs=None):
    """The learner gather of wire-encoded observations (SPEC §8c, nmmo_amd.wire): every rank's
    packed buffer reaches rank `dst`, each peer -> root transfer carrying exactly the bytes its
    header announces (a fixed-size header first, then the payload). Returns, on `dst`, the
    buffers in rank order (dst's own `wire` in place, no self-copy); None elsewhere.
    `recv_bufs[r]` (dst only) holds rank r's buffer (nmmo_wire_max_bytes of its shard); they are
    allocated when missing. The sender reads its total size on the host (one 8-byte copy)."""
    world, rank = dist.get_world_size(), dist.get_rank()
    if world == 1:
        return [wire]

    def total_of(buf):
        return int(buf[:8].view(torch.int64).item())

    if rank != dst:
        total = total_of(wire)
        reqs = [dist.isend(wire[:header_bytes], dst)]
        if total > header_bytes:
            reqs.append(dist.isend(wire[header_bytes:total], dst))
        for q in reqs:
            q.wait()
        return None
    bufs = list(recv_bufs) if recv_bufs is not None else [None] * world
    peers = [r for r in range(world) if r != dst]
    for r in peers:
        if bufs[r] is None:
            bufs[r] = torch.empty_like(wire)
    for q in [dist.irecv(bufs[r][:header_bytes], src=r) for r in peers]:
        q.wait()
    totals = {r: total_of(bufs[r]) for r in peers}
    reqs = [dist.irecv(bufs[r][header_bytes:totals[r]], src=r) for r in peers if totals[r] > header_bytes]
    for q in reqs:
        q.wait()
    bufs[dst] = wire
    return [bufs[r][:totals[r]] if r != dst else wire for r in range(world)]
