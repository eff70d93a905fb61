"""Wire encoding (SPEC.md §8c) on the CPU: the numpy restatement (oracle/wire.py) round-trips the
native layout bit-exactly and shrinks it, and the learner-gather protocol
(nmmo_amd.distributed.WireExchange: each step's sizes, then exactly the announced payload one
step behind) delivers every rank's buffers to the root over gloo (world size 2)."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from nmmo_amd import abi
from nmmo_amd.config import Config
from oracle import wire as owire
from oracle.oracle import OracleEnvs, split_state
from tests.test_native_layout import encode_native


def _native(n_envs, ticks, seed=4, env_index_base=0, with_gold=False):
    cfg = Config.preset("C4", MAP_N=4, early_stop_agent_num=8)
    orc = OracleEnvs(cfg, n_envs, seed=seed, env_index_base=env_index_base)
    orc.reset()
    for t in range(ticks):
        orc.step(orc.scripted_actions(t))
    task = np.arange(n_envs * cfg.PLAYER_N).reshape(n_envs, cfg.PLAYER_N) % 5
    nat = encode_native(orc.obs, cfg.PLAYER_N, task.astype(np.int16))
    if not with_gold:
        return nat, cfg.PLAYER_N
    gold = split_state(orc.get_state(), n_envs, orc.S, orc.P)["ent"][:, abi.F["gold"], :orc.P]
    return nat, cfg.PLAYER_N, gold


def test_wire_roundtrip_and_size():
    nat, P, gold = _native(3, 40, with_gold=True)
    w = owire.pack(nat, P, gold)
    assert int(w[:8].view(np.int64)[0]) == w.nbytes
    back = owire.unpack(w, 3, P)
    assert np.array_equal(back, nat)
    cnt, nm = owire.counts(nat, P)
    assert (cnt & 0x8000).any() and nm.sum() > 0  # agents in the realm and listings were exercised
    assert w.nbytes * 4 < nat.nbytes, (w.nbytes, nat.nbytes)


def test_wire_entity_table():
    """v3: each env's entity table holds every distinct Entity row its records show exactly once,
    ascending by the id's 16-bit pattern, and every record's indices select its own rows; an
    entity seen by several agents makes the buffer smaller than inline rows would."""
    nat, P, gold = _native(3, 50, seed=6, with_gold=True)
    w = owire.pack(nat, P, gold)
    n = 3
    env_off = w[8:8 + 8 * n].copy().view(np.int64)
    o = 8 + 8 * n
    cnt = w[o:o + 2 * n * P].copy().view(np.uint16).reshape(n, P)
    ne = w[o + 2 * n * P + 2 * n:o + 2 * n * P + 4 * n].copy().view(np.uint16)
    _, i16, _ = owire._rows(nat, P)
    shown = inline = 0
    for e in range(n):
        table = w[int(env_off[e]):int(env_off[e]) + 62 * int(ne[e])].copy().view(np.int16).reshape(-1, owire.NE)
        ids = table[:, 0].astype(np.int64) & 0xFFFF
        assert np.all(np.diff(ids) > 0)  # unique, ascending by the 16-bit pattern
        pos = int(env_off[e]) + owire.table_bytes(int(ne[e]))
        seen = set()
        for a in range(P):
            c = int(cnt[e, a])
            if not c & 0x8000:
                continue
            nv = c & 127
            idx = w[pos + owire.HEAD:pos + owire.HEAD + 2 * nv].copy().view(np.uint16)
            rows = i16[e, a, owire.I16_ENTITY:owire.I16_ENTITY + owire.NE * nv].reshape(-1, owire.NE)
            assert np.array_equal(table[idx], rows)
            seen.update(idx.tolist())
            shown += nv
            pos += owire.record_bytes(c)
        assert seen == set(range(int(ne[e])))  # no row the records do not show
        inline += int(ne[e])
    assert shown > inline  # entities shared between agents travel once


def test_wire_buy_mask_is_rebuilt_from_the_listings():
    """Buy.MarketItem is not sent: unpack rebuilds it from the env's listings, the head's gold
    and the agent id (an agent can buy a listing it can afford and does not own), so a record
    with a changed gold decodes to the mask of that gold."""
    nat, P, gold = _native(3, 60, seed=5, with_gold=True)
    cnt, nm = owire.counts(nat, P)
    assert nm.max() > 0, "listings exercised"
    e = int(np.argmax(nm))
    rich = gold.copy()
    rich[e] = 10_000
    back = owire.unpack(owire.pack(nat, P, rich), 3, P)
    rows = back[e, :P * abi.NATIVE_ROW_BYTES].reshape(P, abi.NATIVE_ROW_BYTES)
    market = back[e, P * abi.NATIVE_ROW_BYTES:].copy().view(np.int16).reshape(abi.MARKET_ROWS, 16)
    for a in np.nonzero(cnt[e] & 0x8000)[0]:
        buy = rows[a, owire.BUY_LO:owire.BUY_LO + owire.BUY_N]
        want = (np.arange(owire.BUY_N - 1) < nm[e]) & (market[:, 2] != a + 1)
        assert np.array_equal(buy[:-1], want.astype(np.uint8)) and buy[-1] == 1


def test_wire_all_dead_env():
    nat, P, gold = _native(2, 5, with_gold=True)
    nat[1] = 0  # an env with nobody in the realm and no listings
    w = owire.pack(nat, P, gold)
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
    nat, P, gold = _native(n, 8 + 5 * t + 7 * rank, seed=9, env_index_base=rank * n, with_gold=True)
    small = (np.arange(n * P * 8) * (rank + 3) + t).astype(np.uint8)
    return owire.pack(nat, P, gold), small, P


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


def _fail_worker(rank, world, port, q, mode):
    """Rank 1 announces a tick fault word (mode "fault") or an impossible wire size (mode
    "size") for step 1; every rank must raise at payload(1), before posting its transfers."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from nmmo_amd import distributed as nd
    from nmmo_amd.engine import TickFault

    n, ring = 2, 3
    P = Config.preset("C4").PLAYER_N
    cap = owire.header_bytes(n, P) + n * (P * 9552 + abi.NATIVE_MARKET_BYTES)
    x = nd.WireExchange(world, rank, 1, [cap], [n * P * 8], torch.device("cpu"), ring=ring, backend="gloo")
    wires = [torch.zeros(cap, dtype=torch.uint8) for _ in range(ring)]
    smalls = [torch.zeros(n * P * 8, dtype=torch.uint8) for _ in range(ring)]
    outcome = "no error"
    try:
        for t in range(3):
            w, sm, _ = _step_bytes(rank, t, n)
            wires[t % ring][:w.nbytes] = torch.from_numpy(w)
            smalls[t % ring][:] = torch.from_numpy(sm)
            fault = torch.zeros(1, dtype=torch.int32)
            if rank == 1 and t == 1:
                if mode == "fault":
                    fault[0] = 1 | 5 << 8
                else:
                    wires[t % ring][:8] = torch.tensor([cap + 1], dtype=torch.int64).view(torch.uint8)
            if t >= 1:
                x.post_payload(t - 1, [wires[(t - 1) % ring]], [smalls[(t - 1) % ring]])
            x.post_sizes(t, [wires[t % ring]], fault=fault)
            assert not fault.any()  # zeroed once shipped
        x.post_payload(2, [wires[2]], [smalls[2]])
    except TickFault as err:
        outcome = f"TickFault {err.code} {err.env} step1={'step 1' in str(err)}"
    except RuntimeError as err:
        outcome = f"RuntimeError step1={'step 1' in str(err)}"
    q.put((rank, outcome))
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["fault", "size"])
def test_wire_gather_fails_on_both_ends_without_hanging(mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_fail_worker, args=(r, 2, port, q, mode)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=300)
        assert p.exitcode == 0
    got = dict(q.get(timeout=10) for _ in range(2))
    want = "TickFault 1 5 step1=True" if mode == "fault" else "RuntimeError step1=True"
    assert got == {0: want, 1: want}
