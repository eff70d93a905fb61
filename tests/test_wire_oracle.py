"""Wire encoding (SPEC.md §8c) on the CPU: the numpy restatement (oracle/wire.py) round-trips the
native layout bit-exactly and shrinks it, and the learner-gather protocol
(nmmo_amd.distributed.WireExchange: each step's sizes, then exactly the announced payload one
step behind) delivers every rank's buffers to the root over gloo (world size 2)."""

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


def _step_bytes(rank, t, n):
    """What rank `rank` sends at step t: an oracle-made wire buffer (its size varies with the
    tick) and a small companion buffer."""
    nat, P = _native(n, 8 + 5 * t + 7 * rank, seed=9, env_index_base=rank * n)
    small = (np.arange(n * P * 8) * (rank + 3) + t).astype(np.uint8)
    return owire.pack(nat, P), small, P


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from nmmo_amd import distributed as nd

    n, steps, ring = 2, 4, 3
    P = Config.preset("C4").PLAYER_N
    cap = owire.header_bytes(n, P) + n * (P * 9552 + abi.NATIVE_MARKET_BYTES)
    x = nd.WireExchange(world, rank, 1, [cap], [n * P * 8], torch.device("cpu"), ring=ring, backend="gloo")
    wires = [torch.zeros(cap, dtype=torch.uint8) for _ in range(ring)]
    smalls = [torch.zeros(n * P * 8, dtype=torch.uint8) for _ in range(ring)]
    received = {}

    def payload(s):
        got = x.post_payload(s, [wires[s % ring]], [smalls[s % ring]])
        for key, (w, sm) in got.items():
            received[s, key[0]] = (w.numpy().copy(), sm.numpy().copy())

    # the lagged schedule of WireGather.step: step t's sizes, step t - 1's payload
    for t in range(steps):
        w, sm, _ = _step_bytes(rank, t, n)
        wires[t % ring][:w.nbytes] = torch.from_numpy(w)
        wires[t % ring][w.nbytes:w.nbytes + 64] = 0xAB  # bytes past the total never travel
        smalls[t % ring][:] = torch.from_numpy(sm)
        if t >= 1:
            payload(t - 1)
        x.post_sizes(t, [wires[t % ring]])
    payload(steps - 1)
    if rank == 0:
        ok = len(received) == steps * world
        for t in range(steps):
            for r in range(world):
                w, sm, _ = _step_bytes(r, t, n)
                gw, gs = received[t, r]
                ok &= np.array_equal(gw, w) and np.array_equal(gs, sm)
                ok &= np.array_equal(owire.unpack(gw, n, P), owire.unpack(w, n, P))
        ok &= x.payload_bytes == sum(_step_bytes(r, t, n)[0].nbytes for t in range(steps) for r in range(1, world))
        q.put(bool(ok))
    dist.destroy_process_group()


def test_wire_gather_protocol_gloo():
    """WireExchange over gloo (world size 2, CPU tensors): the lagged protocol (step t's sizes,
    then step t - 1's payload of exactly the announced bytes) delivers every rank's buffers of
    every step to the root bit-exactly, its own in place."""
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
