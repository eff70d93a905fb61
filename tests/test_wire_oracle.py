"""Wire encoding (SPEC.md §8c) on the CPU: the numpy restatement (oracle/wire.py) round-trips the
native layout bit-exactly and shrinks it, and the learner-gather protocol
(nmmo_amd.distributed.gather_wire_to_learner: fixed header, then exactly the announced payload)
delivers every rank's buffer to the root over gloo (world size 2)."""

import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from nmmo_amd import abi
from nmmo_amd.config import Config
from oracle import wire as owire
from oracle.oracle import OracleEnvs
from tests.test_native_layout import encode_native


def _native(n_envs, ticks, seed=4, env_index_base=0):
    cfg = Config.preset("C4", MAP_N=4, early_stop_agent_num=8)
    orc = OracleEnvs(cfg, n_envs, seed=seed, env_index_base=env_index_base)
    orc.reset()
    for t in range(ticks):
        orc.step(orc.scripted_actions(t))
    task = np.arange(n_envs * cfg.PLAYER_N).reshape(n_envs, cfg.PLAYER_N) % 5
    return encode_native(orc.obs, cfg.PLAYER_N, task.astype(np.int16)), cfg.PLAYER_N


def test_wire_roundtrip_and_size():
    nat, P = _native(3, 40)
    w = owire.pack(nat, P)
    assert int(w[:8].view(np.int64)[0]) == w.nbytes
    back = owire.unpack(w, 3, P)
    assert np.array_equal(back, nat)
    cnt, nm = owire.counts(nat, P)
    assert (cnt & 0x8000).any() and nm.sum() > 0  # agents in the realm and listings were exercised
    assert w.nbytes * 4 < nat.nbytes, (w.nbytes, nat.nbytes)


def test_wire_all_dead_env():
    nat, P = _native(2, 5)
    nat[1] = 0  # an env with nobody in the realm and no listings
    w = owire.pack(nat, P)
    assert np.array_equal(owire.unpack(w, 2, P), nat)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from nmmo_amd import distributed as nd

    n = 2
    nat, P = _native(n, 30 + 7 * rank, seed=9, env_index_base=rank * n)
    packed = owire.pack(nat, P)
    cap = owire.header_bytes(n, P) + n * (P * 9552 + abi.NATIVE_MARKET_BYTES)
    buf = torch.zeros(cap, dtype=torch.uint8)
    buf[:packed.nbytes] = torch.from_numpy(packed)
    got = nd.gather_wire_to_learner(buf, owire.header_bytes(n, P))
    if rank == 0:
        ok = True
        for r in range(world):
            ref, _ = _native(n, 30 + 7 * r, seed=9, env_index_base=r * n)
            w = got[r].numpy()
            ok &= np.array_equal(owire.unpack(w, n, P), ref)
        q.put(bool(ok))
    dist.destroy_process_group()


def test_wire_gather_protocol_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=300)
        assert p.exitcode == 0
    assert q.get(timeout=10)
