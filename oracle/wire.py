"""numpy restatement of the wire encoding (SPEC.md §8c) — TEST INFRASTRUCTURE ONLY.

Checker for nmmo_amd/csrc/wire.hip. It derives every count from the native bytes themselves
(an agent is in the realm iff its AgentId is non-zero; nv = Entity rows with a non-zero id;
ninv = Inventory rows with a non-zero item row; listings = Market rows with a non-zero item
row), where the HIP path takes them from the obs kernel. The record head carries the agent's
gold and the Exchange flag (state, not native bytes: the caller passes them); Buy.MarketItem is
not sent and unpack rebuilds it from the listings. Each env's distinct Entity rows travel once,
in its entity table (ascending by the 16-bit pattern of the id), and a record holds the table
index of each of its rows (v3). Never imported by the product path.
"""

from __future__ import annotations

import numpy as np

from nmmo_amd import abi

HEAD, MASK, TILES = 16, 80, 113        # the mask without Buy.MarketItem; 4-bit materials
BUY_LO, BUY_N, MASK_N = 104, 1025, 1586
SENT = np.r_[0:BUY_LO, BUY_LO + BUY_N:MASK_N]  # flat mask entries a record carries, in bit order
I16_ENTITY, NE = 2, 31
I16_INV = I16_ENTITY + 100 * NE
I16_TILE = I16_INV + 12 * 16
I16_TASK = I16_TILE + 225 * 3


def header_bytes(n: int, P: int) -> int:
    return (8 + 8 * n + 2 * n * P + 4 * n + 15) & ~15


def record_bytes(cnt: int) -> int:
    if not cnt & 0x8000:
        return 0
    nv, ninv = cnt & 127, (cnt >> 7) & 15
    return (HEAD + MASK + 2 * nv + 32 * ninv + TILES + 15) & ~15


def table_bytes(ne: int) -> int:
    return (62 * ne + 15) & ~15


def _rows(native: np.ndarray, P: int):
    n = native.shape[0]
    rows = native[:, :P * abi.NATIVE_ROW_BYTES].reshape(n, P, abi.NATIVE_ROW_BYTES)
    i16 = rows[:, :, abi.NATIVE_MASK_BYTES:].copy().view(np.int16)
    market = native[:, P * abi.NATIVE_ROW_BYTES:].copy().view(np.int16).reshape(n, abi.MARKET_ROWS, 16)
    return rows, i16, market


def counts(native: np.ndarray, P: int):
    rows, i16, market = _rows(native, P)
    ent_ids = i16[:, :, I16_ENTITY:I16_INV].reshape(*i16.shape[:2], 100, NE)[..., 0]
    inv_rows = i16[:, :, I16_INV:I16_TILE].reshape(*i16.shape[:2], 12, 16)[..., 0]
    nv = (ent_ids != 0).sum(-1)
    ninv = (inv_rows != 0).sum(-1)
    alive = i16[:, :, 0] != 0
    cnt = np.where(alive, 0x8000 | nv | (ninv << 7), 0).astype(np.uint16)
    nm = (market[:, :, 0] != 0).sum(-1).astype(np.uint16)
    return cnt, nm


def listing_offset(cnt_env, ne: int) -> int:
    """Offset of an env's listings in its payload: its entity table and records."""
    return table_bytes(ne) + sum(record_bytes(int(c)) for c in cnt_env)


def _table(i16e: np.ndarray, cnt_e: np.ndarray):
    """One env's entity table: {id: row} over its records' Entity rows, and the ids in table
    order (ascending by the id's 16-bit pattern)."""
    rows = {}
    for a, c in enumerate(cnt_e):
        c = int(c)
        if not c & 0x8000:
            continue
        ent = i16e[a, I16_ENTITY:I16_ENTITY + NE * (c & 127)].reshape(-1, NE)
        for r in ent:
            rows.setdefault(int(r[0]), r)
    order = sorted(rows, key=lambda i: i & 0xFFFF)
    return rows, order


def pack(native: np.ndarray, P: int, gold: np.ndarray, exch: bool = True) -> np.ndarray:
    """native uint8 [n, env_bytes] -> wire uint8 [total]; gold int [n, P] = each agent's gold in
    the state the obs was taken from."""
    n = native.shape[0]
    rows, i16, market = _rows(native, P)
    cnt, nm = counts(native, P)
    tables = [_table(i16[e], cnt[e]) for e in range(n)]
    ne = np.array([len(t[1]) for t in tables], np.uint16)
    H = header_bytes(n, P)
    env_bytes = [listing_offset(cnt[e], int(ne[e])) + 32 * int(nm[e]) for e in range(n)]
    env_off = np.cumsum([H] + env_bytes)
    total = int(env_off[-1])
    out = np.zeros(total, np.uint8)
    out[:8] = np.array([total], np.int64).view(np.uint8)
    out[8:8 + 8 * n] = env_off[:-1].astype(np.int64).view(np.uint8)
    o = 8 + 8 * n
    out[o:o + 2 * n * P] = cnt.reshape(-1).view(np.uint8)
    out[o + 2 * n * P:o + 2 * n * P + 2 * n] = nm.view(np.uint8)
    out[o + 2 * n * P + 2 * n:o + 2 * n * P + 4 * n] = ne.view(np.uint8)
    for e in range(n):
        pos = int(env_off[e])
        trows, order = tables[e]
        index = {i: k for k, i in enumerate(order)}
        if order:
            out[pos:pos + 62 * len(order)] = np.stack([trows[i] for i in order]).astype(np.int16).view(np.uint8).reshape(-1)
        pos += table_bytes(len(order))
        for a in range(P):
            c = int(cnt[e, a])
            if not c & 0x8000:
                continue
            nv, ninv = c & 127, (c >> 7) & 15
            q = i16[e, a]
            head = np.array([q[0], q[1], q[I16_TASK], q[I16_TILE], q[I16_TILE + 1], nv, ninv | (int(exch) << 8),
                             gold[e, a]], np.int16)
            rec = np.zeros(record_bytes(c), np.uint8)
            rec[:HEAD] = head.view(np.uint8)
            bits = np.packbits(rows[e, a, SENT] != 0, bitorder="little")
            rec[HEAD:HEAD + len(bits)] = bits
            k = HEAD + MASK
            ids = q[I16_ENTITY:I16_ENTITY + NE * nv].reshape(-1, NE)[:, 0]
            rec[k:k + 2 * nv] = np.array([index[int(i)] for i in ids], np.uint16).view(np.uint8)
            k += 2 * nv
            rec[k:k + 32 * ninv] = q[I16_INV:I16_INV + 16 * ninv].view(np.uint8)
            k += 32 * ninv
            mats = np.zeros(2 * TILES, np.uint8)
            mats[:225] = q[I16_TILE + 2:I16_TASK:3].astype(np.uint8) & 15
            rec[k:k + TILES] = mats[0::2] | (mats[1::2] << 4)
            out[pos:pos + len(rec)] = rec
            pos += len(rec)
        out[pos:pos + 32 * int(nm[e])] = market[e, :int(nm[e])].reshape(-1).view(np.uint8)
    return out


def unpack(wire: np.ndarray, n: int, P: int) -> np.ndarray:
    """wire uint8 -> native uint8 [n, env_bytes]."""
    out = np.zeros((n, abi.native_env_bytes(P)), np.uint8)
    env_off = wire[8:8 + 8 * n].copy().view(np.int64)
    o = 8 + 8 * n
    cnt = wire[o:o + 2 * n * P].copy().view(np.uint16).reshape(n, P)
    nm = wire[o + 2 * n * P:o + 2 * n * P + 2 * n].copy().view(np.uint16)
    ne = wire[o + 2 * n * P + 2 * n:o + 2 * n * P + 4 * n].copy().view(np.uint16)
    for e in range(n):
        pos = int(env_off[e])
        table = wire[pos:pos + 62 * int(ne[e])].copy().view(np.int16).reshape(-1, NE)
        pos += table_bytes(int(ne[e]))
        for a in range(P):
            c = int(cnt[e, a])
            if not c & 0x8000:
                continue
            nv, ninv = c & 127, (c >> 7) & 15
            rec = wire[pos:pos + record_bytes(c)]
            pos += len(rec)
            head = rec[:HEAD].copy().view(np.int16)
            row = out[e, a * abi.NATIVE_ROW_BYTES:(a + 1) * abi.NATIVE_ROW_BYTES]
            row[SENT] = np.unpackbits(rec[HEAD:HEAD + MASK], bitorder="little")[:len(SENT)]
            # Buy.MarketItem: listing k < nm is buyable iff Exchange, price <= gold, owner != self
            buy = np.zeros(BUY_N, np.uint8)
            buy[BUY_N - 1] = 1
            nmk = int(nm[e])
            if nmk and (int(head[6]) >> 8) & 1:
                lo = int(env_off[e]) + listing_offset(cnt[e], int(ne[e]))
                lst = wire[lo:lo + 32 * nmk].copy().view(np.int16).reshape(nmk, 16)
                buy[:nmk] = (lst[:, 15] <= head[7]) & (lst[:, 2] != head[0])
            row[BUY_LO:BUY_LO + BUY_N] = buy
            q = np.zeros(abi.NATIVE_I16, np.int16)
            q[0], q[1] = head[0], head[1]
            k = HEAD + MASK
            idx = rec[k:k + 2 * nv].copy().view(np.uint16)
            q[I16_ENTITY:I16_ENTITY + NE * nv] = table[idx].reshape(-1)
            k += 2 * nv
            q[I16_INV:I16_INV + 16 * ninv] = rec[k:k + 32 * ninv].copy().view(np.int16)
            k += 32 * ninv
            t = np.arange(225)
            q[I16_TILE:I16_TASK:3] = head[3] + t // 15
            q[I16_TILE + 1:I16_TASK:3] = head[4] + t % 15
            mats = np.stack([rec[k:k + TILES] & 15, rec[k:k + TILES] >> 4], 1).reshape(-1)[:225]
            q[I16_TILE + 2:I16_TASK:3] = mats
            q[I16_TASK] = head[2]
            row[abi.NATIVE_MASK_BYTES:] = q.view(np.uint8)
        mk = out[e, P * abi.NATIVE_ROW_BYTES:]
        mk[:32 * int(nm[e])] = wire[pos:pos + 32 * int(nm[e])]
    return out
