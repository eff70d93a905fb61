"""Multi-rank path on CPU (gloo, world_size 2): envs sharded by global index, actions scattered
from the learner, outputs gathered back. The sharded run must equal a single-process run of
the same total envs env-for-env (the property the 8-GPU bench relies on). The per-rank stepper
here is the CPU oracle (test stand-in for the HIP engine, same API)."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from nmmo_amd import distributed as nd
from nmmo_amd.config import Config

TOTAL, STEPS = 4, 12


def _cfg():
    return Config.preset("C4", MAP_N=2, early_stop_agent_num=8)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, reset_seed=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle.oracle import OracleEnvs

    base, n = nd.shard(TOTAL, world, rank)
    from nmmo_amd.vecenv import reset_seeds

    o = OracleEnvs(_cfg(), n, seed=31, env_index_base=base)
    # GpuVecEnv.async_reset(seed)'s per-env seeds for this shard (clean_pufferl.py:175)
    o.reset(None if reset_seed is None else reset_seeds(reset_seed, base, n))
    results = []
    full_ref = None
    if rank == 0:
        full_ref = OracleEnvs(_cfg(), TOTAL, seed=31)
        full_ref.reset(None if reset_seed is None else reset_seeds(reset_seed, 0, TOTAL))
    for t in range(STEPS):
        full_a = torch.from_numpy(full_ref.scripted_actions(100 + t)) if rank == 0 else None
        local_a = nd.scatter_from_learner(full_a, torch.zeros((n, o.P, 12), dtype=torch.int32))
        # the rank's own policy stream agrees with the learner's slice (global env indices)
        assert np.array_equal(local_a.numpy(), o.scripted_actions(100 + t))
        o.step(local_a.numpy())
        outs = [nd.gather_to_learner(torch.from_numpy(x.copy()))
                for x in (o.obs, o.rew, o.term, o.trunc, o.mask)]
        if rank == 0:
            full_ref.step(full_a.numpy())
            ok = all(np.array_equal(g.numpy(), r) for g, r in
                     zip(outs, (full_ref.obs, full_ref.rew, full_ref.term, full_ref.trunc, full_ref.mask)))
            results.append(ok)
    if rank == 0:
        q.put(results)
    dist.destroy_process_group()


@pytest.mark.parametrize("reset_seed", [None, 42])
def test_sharded_equals_single_process(reset_seed):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, reset_seed)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert len(res) == STEPS and all(res)


def test_reset_seeds_distinct_across_shards():
    from nmmo_amd.vecenv import reset_seeds

    a = np.concatenate([reset_seeds(7, r * 4, 4) for r in range(2)])
    assert np.array_equal(a, reset_seeds(7, 0, 8))
    assert len(set(a.tolist())) == 8


def test_shard_bounds():
    assert nd.shard(8192, 8, 3) == (3072, 1024)
    try:
        nd.shard(10, 4, 0)
    except ValueError:
        pass
    else:
        raise AssertionError("uneven split must raise")


def test_env_shares_learner_split():
    """C5's learner share (bench.py --root-envs): rank 0 holds root_envs, the peers split the rest
    as evenly as possible in whole env batches, and the node still steps every env."""
    assert nd.env_shares(8192, 8, 512, granule=2) == [512] + [1098] * 4 + [1096] * 3
    for world, k in ((2, 896), (4, 640), (8, 256), (8, 1024)):
        sh = nd.env_shares(1024 * world, world, k, granule=2)
        assert sh[0] == k and sum(sh) == 1024 * world
        assert all(n % 2 == 0 for n in sh) and max(sh[1:]) - min(sh[1:]) <= 2
    assert nd.env_shares(4096, 4, None) == [1024] * 4
    assert nd.env_shares(1024, 1, 100) == [1024]
    with pytest.raises(ValueError):
        nd.env_shares(1024 * 8, 8, 511, granule=2)
    with pytest.raises(ValueError):
        nd.env_shares(16, 8, 14, granule=2)
