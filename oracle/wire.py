"""numpy restatement of the wire encoding (SPEC.md §8c) — TEST INFRASTRUCTURE ONLY.

Checker for nmmo_amd/csrc/wire.hip. It derives every count from the native bytes themselves
(an agent is in the realm iff its AgentId is non-zero; nv = Entity rows with a non-zero id;
ninv = Inventory rows with a non-zero item row; listings = Market rows with a non-zero item
row), where the HIP path takes them from the obs kernel. The record head carries the agent's
gold and the Exchange flag (state, not native bytes: the caller passes them); Buy.MarketItem is
not sent and unpack rebuilds it from the listings. Each env's distinct Entity rows travel once,
in its entity table (ascending by the 16-bit pattern of the id), and a record holds the table
index of each of its rows (v3). v4: the other ActionTargets sections travel as what they are made
of -- Style and Move in the head, GoldPrice as its count of leading ones, SellPrice as the price
the wrapper cleared (+1, 0 = none), and only the first nv entries of the three target sections
and the first ninv of the four inventory sections as a bit stream at the record's end (every
entry past them is 0 and each noop entry 1). Never imported by the product path.
"""

from __future__ import annotations

import numpy as np

from nmmo_amd import abi

HEAD, TILES = 16, 114                  # 4-bit materials (225 nibbles + a zero nibble and a zero byte)
BUY_LO, BUY_N, MASK_N = 104, 1025, 1586
# ActionTargets sections in flat order: (flat offset, entries)
STYLE, ATTACK_T, BUY, DESTROY, GIVE_I, GIVE_T, GOLD_P, GOLD_T, MOVE, SELL_I, SELL_P, USE = (
    (0, 3), (3, 101), (104, 1025), (1129, 13), (1142, 13), (1155, 101), (1256, 99), (1355, 101), (1456, 5),
    (1461, 13), (1474, 99), (1573, 13))
TARGETS = (ATTACK_T, GIVE_T, GOLD_T)     # stream order: nv entries each, then
INVENTORY = (DESTROY, GIVE_I, SELL_I, USE)  # ninv entries each
I16_ENTITY, NE = 2, 31
I16_INV = I16_ENTITY + 100 * NE
I16_TILE = I16_INV + 12 * 16
I16_TASK = I16_TILE + 225 * 3


def header_bytes(n: int, P: int) -> int:
    return (8 + 8 * n + 2 * n * P + 4 * n + 15) & ~15


def stream_bytes(nv: int, ninv: int) -> int:
    """The mask bit stream's bytes: 3 nv + 4 ninv bits in whole 16-bit words."""
    return 2 * ((3 * nv + 4 * ninv + 15) // 16)


def record_bytes(cnt: int) -> int:
    if not cnt & 0x8000:
        return 0
    nv, ninv = cnt & 127, (cnt >> 7) & 15
    return (HEAD + 2 * nv + 32 * ninv + TILES + stream_bytes(nv, ninv) + 15) & ~15


def head_mask_words(row: np.ndarray, nv: int, ninv: int, exch: bool):
    """Head words 5 and 6 (SPEC §8c v4) from a native row's mask bytes: nv | ninv << 7 | Exchange
    << 11 | (pp1 & 15) << 12 and Style | Move << 1 | GoldPrice count << 6 | (pp1 >> 4) << 13, where
    pp1 = 1 + the SellPrice entry the wrapper cleared (0 = none)."""
    m = row[:MASK_N] != 0
    style = int(m[STYLE[0]])
    move = int(np.packbits(m[MOVE[0]:MOVE[0] + 5], bitorder="little")[0])
    ng = int(m[GOLD_P[0]:GOLD_P[0] + GOLD_P[1]].sum())
    sp = m[SELL_P[0]:SELL_P[0] + SELL_P[1]]
    pp1 = 0
    if exch and not sp.all():
        pp1 = int(np.flatnonzero(~sp)[0]) + 1
    h5 = nv | ninv << 7 | int(exch) << 11 | (pp1 & 15) << 12
    h6 = style | move << 1 | ng << 6 | (pp1 >> 4) << 13
    return np.array([h5, h6], np.uint16).view(np.int16)


def stream_bits(row: np.ndarray, nv: int, ninv: int) -> np.ndarray:
    """The record's mask bit stream (little-endian bit order, zero-padded to stream_bytes)."""
    m = row[:MASK_N] != 0
    bits = [m[o:o + nv] for o, _ in TARGETS] + [m[o:o + ninv] for o, _ in INVENTORY]
    out = np.zeros(stream_bytes(nv, ninv), np.uint8)
    b = np.packbits(np.concatenate(bits), bitorder="little") if nv or ninv else np.zeros(0, np.uint8)
    out[:len(b)] = b
    return out


def mask_from_record(head: np.ndarray, stream: np.ndarray, nv: int, ninv: int) -> np.ndarray:
    """The 1,586 ActionTargets entries of a record, Buy.MarketItem left 0."""
    h5, h6 = int(head[5]) & 0xFFFF, int(head[6]) & 0xFFFF
    exch = (h5 >> 11) & 1
    pp1 = (h5 >> 12) | (h6 >> 13) << 4
    m = np.zeros(MASK_N, np.uint8)
    m[STYLE[0]:STYLE[0] + 3] = h6 & 1
    m[MOVE[0]:MOVE[0] + 5] = [(h6 >> (1 + k)) & 1 for k in range(5)]
    ng = (h6 >> 6) & 127
    m[GOLD_P[0]:GOLD_P[0] + ng] = 1
    if exch:
        m[SELL_P[0]:SELL_P[0] + SELL_P[1]] = 1
        if pp1:
            m[SELL_P[0] + pp1 - 1] = 0
    bits = np.unpackbits(stream, bitorder="little")
    k = 0
    for o, n in TARGETS:
        m[o:o + nv] = bits[k:k + nv]
        m[o + n - 1] = 1  # noop
        k += nv
    for o, n in INVENTORY:
        m[o:o + ninv] = bits[k:k + ninv]
        m[o + n - 1] = 1
        k += ninv
    return m


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
            h56 = head_mask_words(rows[e, a], nv, ninv, exch)
            head = np.array([q[0], q[1], q[I16_TASK], q[I16_TILE], q[I16_TILE + 1], h56[0], h56[1], gold[e, a]],
                            np.int16)
            rec = np.zeros(record_bytes(c), np.uint8)
            rec[:HEAD] = head.view(np.uint8)
            k = HEAD
            ids = q[I16_ENTITY:I16_ENTITY + NE * nv].reshape(-1, NE)[:, 0]
            rec[k:k + 2 * nv] = np.array([index[int(i)] for i in ids], np.uint16).view(np.uint8)
            k += 2 * nv
            rec[k:k + 32 * ninv] = q[I16_INV:I16_INV + 16 * ninv].view(np.uint8)
            k += 32 * ninv
            mats = np.zeros(2 * TILES, np.uint8)
            mats[:225] = q[I16_TILE + 2:I16_TASK:3].astype(np.uint8) & 15
            rec[k:k + TILES] = mats[0::2] | (mats[1::2] << 4)
            k += TILES
            st = stream_bits(rows[e, a], nv, ninv)
            rec[k:k + len(st)] = st
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
            so = HEAD + 2 * nv + 32 * ninv + TILES
            row[:MASK_N] = mask_from_record(head, rec[so:so + stream_bytes(nv, ninv)], nv, ninv)
            # Buy.MarketItem: listing k < nm is buyable iff Exchange, price <= gold, owner != self
            buy = np.zeros(BUY_N, np.uint8)
            buy[BUY_N - 1] = 1
            nmk = int(nm[e])
            if nmk and (int(head[5]) >> 11) & 1:
                lo = int(env_off[e]) + listing_offset(cnt[e], int(ne[e]))
                lst = wire[lo:lo + 32 * nmk].copy().view(np.int16).reshape(nmk, 16)
                buy[:nmk] = (lst[:, 15] <= head[7]) & (lst[:, 2] != head[0])
            row[BUY_LO:BUY_LO + BUY_N] = buy
            q = np.zeros(abi.NATIVE_I16, np.int16)
            q[0], q[1] = head[0], head[1]
            k = HEAD
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
