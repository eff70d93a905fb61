"""Observation / action layout of the pufferlib-0.7.3-flattened nmmo 2.1 spaces.

The reference never spells the flat layout out; it consumes it through
`pufferlib.emulation.unpack_batched_obs(flat, env.unflatten_context)`
(agent_zoo/neurips23_start_kit/baseline_policy.py:7,41) and indexes the result by key:
Tile (:96-104), Entity (:118-140), Inventory/Market items (:151-163), Task (:242), AgentId (:43),
ActionTargets (:245-262). pufferlib flattens a Dict space with its keys sorted at every level,
so the flat vector is: ActionTargets{Attack{Style,Target}, Buy{MarketItem}, Destroy{InventoryItem},
Give{InventoryItem,Target}, GiveGold{Price,Target}, Move{Direction}, Sell{InventoryItem,Price},
Use{InventoryItem}}, AgentId, CurrentTick, Entity, Inventory, Market, Task, Tile.
"""

from __future__ import annotations

import collections

import numpy as np

PLAYER_N_OBS = 100      # Entity rows; Attack/Give/GiveGold Target masks are this + noop
INVENTORY_N_OBS = 12    # baseline_policy.py:176
MARKET_N_OBS = 1024
PRICE_N_OBS = 99        # baseline_policy.py:217 (gold_quantity / inventory_price heads)
ITEM_COLS = 16          # baseline_policy.py:151-163
ENTITY_COLS = 31        # baseline_policy.py:118
TILE_ROWS = 225         # 15x15, baseline_policy.py:96-104
TILE_COLS = 3           # (row, col, material_id)
N_MOVE = 5              # baseline_policy.py:215
N_STYLE = 3             # baseline_policy.py:207

# (name, size) in pufferlib flat order
MASK_SEGMENTS = [
    (("Attack", "Style"), N_STYLE),
    (("Attack", "Target"), PLAYER_N_OBS + 1),
    (("Buy", "MarketItem"), MARKET_N_OBS + 1),
    (("Destroy", "InventoryItem"), INVENTORY_N_OBS + 1),
    (("Give", "InventoryItem"), INVENTORY_N_OBS + 1),
    (("Give", "Target"), PLAYER_N_OBS + 1),
    (("GiveGold", "Price"), PRICE_N_OBS),
    (("GiveGold", "Target"), PLAYER_N_OBS + 1),
    (("Move", "Direction"), N_MOVE),
    (("Sell", "InventoryItem"), INVENTORY_N_OBS + 1),
    (("Sell", "Price"), PRICE_N_OBS),
    (("Use", "InventoryItem"), INVENTORY_N_OBS + 1),
]

# MultiDiscrete action heads, same sorted order (takeru/policy.py:293-307)
ACTION_HEADS = [(name, size) for name, size in MASK_SEGMENTS]
ACTION_DIMS = [size for _, size in ACTION_HEADS]
HEAD = {f"{a}.{b}": i for i, ((a, b), _) in enumerate(ACTION_HEADS)}

Segment = collections.namedtuple("Segment", "offset shape dtype")


def flat_layout(task_dim: int = 2048) -> "collections.OrderedDict[str, Segment]":
    """Offsets of every leaf of the flat obs. Leaf dtypes are the nmmo 2.1 space dtypes."""
    out = collections.OrderedDict()
    off = 0
    for (a, b), n in MASK_SEGMENTS:
        out[f"ActionTargets.{a}.{b}"] = Segment(off, (n,), np.int8)
        off += n
    for key, shape, dt in [
        ("AgentId", (1,), np.int16),
        ("CurrentTick", (1,), np.int16),
        ("Entity", (PLAYER_N_OBS, ENTITY_COLS), np.int16),
        ("Inventory", (INVENTORY_N_OBS, ITEM_COLS), np.int16),
        ("Market", (MARKET_N_OBS, ITEM_COLS), np.int16),
        ("Task", (task_dim,), np.float16),
        ("Tile", (TILE_ROWS, TILE_COLS), np.int16),
    ]:
        out[key] = Segment(off, shape, dt)
        off += int(np.prod(shape))
    out["__total__"] = Segment(off, (off,), np.float32)
    return out


def obs_elems(task_dim: int = 2048) -> int:
    return flat_layout(task_dim)["__total__"].offset


def unflatten(flat, task_dim: int = 2048) -> dict:
    """Inverse of the flattening for [..., obs_elems] arrays or tensors — the equivalent of
    pufferlib.emulation.unpack_batched_obs for this layout (returns views, nested dicts)."""
    lay = flat_layout(task_dim)
    batch = tuple(flat.shape[:-1])
    out: dict = {"ActionTargets": {}}
    for key, seg in lay.items():
        if key == "__total__":
            continue
        n = int(np.prod(seg.shape))
        view = flat[..., seg.offset:seg.offset + n].reshape(*batch, *seg.shape)
        parts = key.split(".")
        if parts[0] == "ActionTargets":
            out["ActionTargets"].setdefault(parts[1], {})[parts[2]] = view
        else:
            out[key] = view
    return out
