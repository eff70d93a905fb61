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


def unpack_batched_obs(batched_obs, unflatten_context) -> dict:
    """pufferlib.emulation.unpack_batched_obs with the reference's call signature
    (baseline_policy.py:7,41: `unpack_batched_obs(flat_observations, self.unflatten_context)`),
    for the context GpuVecEnv's driver_env hands the policy (`flat_layout`, an OrderedDict of
    Segments): the nested dict of views the policy indexes -- Tile, Entity, AgentId, Inventory,
    Market, Task and ActionTargets[head][arg] (baseline_policy.py:42-76, 230-262). With pufferlib
    absent the policy's one change is importing this name from here. (pufferlib 0.7.3's own
    decoder is not importable in this image: that it accepts this context is unpinned.)"""
    total = unflatten_context["__total__"].offset
    if batched_obs.shape[-1] != total:
        raise ValueError(f"flat obs have {batched_obs.shape[-1]} elements, the context {total}")
    task = unflatten_context["Task"].shape[0]
    return unflatten(batched_obs, task)


# ---------------------------------------------------------------- native layout (SPEC.md §8b)
NATIVE_I16_FIELDS = [("AgentId", (1,)), ("CurrentTick", (1,)), ("Entity", (PLAYER_N_OBS, ENTITY_COLS)),
                     ("Inventory", (INVENTORY_N_OBS, ITEM_COLS)), ("Tile", (TILE_ROWS, TILE_COLS)),
                     ("TaskIndex", (1,))]


def native_offsets() -> dict:
    """int16 offsets of the agent row's fields (after the 1,600 mask bytes)."""
    out, off = {}, 0
    for name, shape in NATIVE_I16_FIELDS:
        out[name] = (off, shape)
        off += int(np.prod(shape))
    return out


def unflatten_native(native, players: int, task_table, task_dim: int = 2048) -> dict:
    """The native obs of n envs (uint8 [n, native_env_bytes], numpy or torch) decoded into the same
    nested dict `unflatten(flat)` returns for [n*players, obs_elems] — float32 values equal to the
    flat layout's, Market broadcast to the env's agents and Task looked up in `task_table`
    (float32 [n_tasks, task_dim]). The learner-side replacement for unpack_batched_obs
    (baseline_policy.py:41) when the env ships the native layout."""
    from . import abi

    torch_in = not isinstance(native, np.ndarray)
    xp_float = (lambda x: x.float()) if torch_in else (lambda x: x.astype(np.float32))
    n = native.shape[0]
    rows = native[:, :players * abi.NATIVE_ROW_BYTES].reshape(n * players, abi.NATIVE_ROW_BYTES)
    masks = rows[:, :abi.NATIVE_MASK_BYTES]
    if torch_in:
        import torch

        i16 = rows[:, abi.NATIVE_MASK_BYTES:].contiguous().view(dtype=torch.int16)
        mk = native[:, players * abi.NATIVE_ROW_BYTES:].contiguous().view(dtype=torch.int16)
    else:
        i16 = np.ascontiguousarray(rows[:, abi.NATIVE_MASK_BYTES:]).view(np.int16)
        mk = np.ascontiguousarray(native[:, players * abi.NATIVE_ROW_BYTES:]).view(np.int16)
    alive = i16[:, 0] != 0
    out: dict = {"ActionTargets": {}}
    off = 0
    for (a, b), size in MASK_SEGMENTS:
        out["ActionTargets"].setdefault(a, {})[b] = xp_float(masks[:, off:off + size])
        off += size
    for name, (o, shape) in native_offsets().items():
        if name == "TaskIndex":
            continue
        k = int(np.prod(shape))
        out[name] = xp_float(i16[:, o:o + k]).reshape(n * players, *shape)
    market = xp_float(mk).reshape(n, 1, MARKET_N_OBS, ITEM_COLS)
    if torch_in:
        market = market.expand(n, players, MARKET_N_OBS, ITEM_COLS).reshape(n * players, MARKET_N_OBS, ITEM_COLS)
        market = market * alive.view(-1, 1, 1)
        tidx = i16[:, native_offsets()["TaskIndex"][0]].long()
        import torch

        task = torch.as_tensor(task_table, dtype=torch.float32, device=market.device)[tidx] * alive.view(-1, 1)
    else:
        market = np.broadcast_to(market, (n, players, MARKET_N_OBS, ITEM_COLS)).reshape(n * players, MARKET_N_OBS, ITEM_COLS)
        market = market * alive.reshape(-1, 1, 1)
        tidx = i16[:, native_offsets()["TaskIndex"][0]].astype(np.int64)
        task = np.asarray(task_table, np.float32)[tidx] * alive.reshape(-1, 1)
    out["Market"] = market
    out["Task"] = task
    return out
