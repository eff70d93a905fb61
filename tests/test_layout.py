"""Layout facts the reference code hard-codes, checked against the flat
layout of all three implementations (python nmmo_amd.layout, the C-ABI nmmo_layout, the oracle)
and against observations the oracle produces. CPU only."""

import ctypes

import numpy as np
import pytest

from nmmo_amd import abi, layout
from nmmo_amd.config import Config
from oracle.oracle import OracleEnvs, split_state

# agent_zoo/takeru/policy.py:293-307 / baseline_policy.py:205-264: head order and sizes
REF_HEADS = [
    ("attack_style", 3), ("attack_target", 101), ("market_buy", 1025),
    ("inventory_destroy", 13), ("inventory_give_item", 13), ("inventory_give_player", 101),
    ("gold_quantity", 99), ("gold_target", 101), ("move", 5), ("inventory_sell", 13),
    ("inventory_price", 99), ("inventory_use", 13),
]
# baseline_policy.py:245-262: head -> ActionTargets key
REF_HEAD_KEYS = [
    ("Attack", "Style"), ("Attack", "Target"), ("Buy", "MarketItem"),
    ("Destroy", "InventoryItem"), ("Give", "InventoryItem"), ("Give", "Target"),
    ("GiveGold", "Price"), ("GiveGold", "Target"), ("Move", "Direction"),
    ("Sell", "InventoryItem"), ("Sell", "Price"), ("Use", "InventoryItem"),
]
# Entity columns named by the reference policies (takeru/policy.py:121-161,
# baseline_policy.py:118-129, yaofeng/policy.py:145-147)
REF_ENTITY_COLS = [
    "id", "npc_type", "attacker_id", "message", "row", "col", "damage", "time_alive", "freeze",
    "item_level", "latest_combat_tick", "gold", "health", "food", "water",
    "melee_level", "melee_exp", "range_level", "range_exp", "mage_level", "mage_exp",
    "fishing_level", "fishing_exp", "herbalism_level", "herbalism_exp", "prospecting_level",
    "prospecting_exp", "carving_level", "carving_exp", "alchemy_level", "alchemy_exp",
]


def test_config_defaults_match_reference():
    c = Config()
    # config.yaml:76-86 / environment.py:31-49
    assert (c.PLAYER_N, c.NPC_N, c.HORIZON, c.MAP_N, c.MAP_CENTER) == (128, 256, 1024, 256, 128)
    assert (c.TASK_EMBED_DIM, c.COMBAT_SPAWN_IMMUNITY) == (2048, 20)
    assert c.RESOURCE_RESILIENT_POPULATION == 0.2
    assert c.PROVIDE_ACTION_TARGETS and c.PROVIDE_NOOP_ACTION_TARGET
    assert c.PLAYER_DEATH_FOG is None
    assert set(c.systems) == {"Resource", "Combat", "NPC", "Progression", "Item", "Equipment",
                              "Profession", "Exchange"}  # environment.py:14-25 (+Medium/Terrain)


def test_config_from_namespace_like_reference():
    from argparse import Namespace

    ns = Namespace(num_agents=64, num_npcs=128, max_episode_length=512, num_maps=16, map_size=128,
                   task_size=2048, spawn_immunity=10, resilient_population=0.0, death_fog_tick=None)
    c = Config(ns)
    assert (c.PLAYER_N, c.NPC_N, c.HORIZON, c.MAP_N, c.COMBAT_SPAWN_IMMUNITY) == (64, 128, 512, 16, 10)


def test_action_heads_match_reference_policies():
    assert [s for _, s in REF_HEADS] == layout.ACTION_DIMS
    assert [k for k, _ in layout.ACTION_HEADS] == REF_HEAD_KEYS


def test_flat_layout_size_and_keys():
    lay = layout.flat_layout(2048)
    assert layout.obs_elems(2048) == 23987
    sizes = {k: int(np.prod(v.shape)) for k, v in lay.items() if k != "__total__"}
    assert sum(v for k, v in sizes.items() if k.startswith("ActionTargets")) == 1586
    assert sizes["Entity"] == 100 * 31 and sizes["Tile"] == 225 * 3
    assert sizes["Inventory"] == 12 * 16 and sizes["Market"] == 1024 * 16 and sizes["Task"] == 2048
    order = [k.split(".")[0] for k in lay if k != "__total__"]
    top = list(dict.fromkeys(order))
    assert top == sorted(top)  # pufferlib sorted-key flattening


def test_three_layouts_agree(oracle_lib):
    from nmmo_amd import _native

    py = layout.flat_layout(2048)
    lay = _native.layout(Config().to_c())
    assert lay.obs_elems == py["__total__"].offset == oracle_lib.oracle_obs_elems(2048)
    offs = (ctypes.c_int32 * 20)()
    oracle_lib.oracle_flat_offsets(2048, offs)
    names = [f"ActionTargets.{a}.{b}" for a, b in REF_HEAD_KEYS] + [
        "AgentId", "CurrentTick", "Entity", "Inventory", "Market", "Task", "Tile"]
    c_offs = [lay.off_mask_attack_style, lay.off_mask_attack_target, lay.off_mask_buy,
              lay.off_mask_destroy, lay.off_mask_give_item, lay.off_mask_give_target,
              lay.off_mask_givegold_price, lay.off_mask_givegold_target, lay.off_mask_move,
              lay.off_mask_sell_item, lay.off_mask_sell_price, lay.off_mask_use,
              lay.off_agent_id, lay.off_current_tick, lay.off_entity, lay.off_inventory,
              lay.off_market, lay.off_task, lay.off_tile]
    for i, n in enumerate(names):
        assert py[n].offset == c_offs[i] == offs[i], n
    assert list(lay.act_dims) == layout.ACTION_DIMS


def test_entity_columns():
    assert abi.ENTITY_FIELDS[:31] == [
        "id", "npc_type", "row", "col", "damage", "time_alive", "freeze", "item_level",
        "attacker_id", "latest_combat_tick", "message", "gold", "health", "food", "water",
        "melee_level", "melee_exp", "range_level", "range_exp", "mage_level", "mage_exp",
        "fishing_level", "fishing_exp", "herbalism_level", "herbalism_exp",
        "prospecting_level", "prospecting_exp", "carving_level", "carving_exp",
        "alchemy_level", "alchemy_exp"]
    assert abi.F["id"] == 0 and abi.F["npc_type"] == 1  # baseline_policy.py:118-119
    assert set(REF_ENTITY_COLS) == set(abi.ENTITY_FIELDS[:31])


@pytest.fixture(scope="module")
def rollout():
    cfg = Config.preset("C4", MAP_N=4, early_stop_agent_num=0)
    task = np.load("tests/golden/task_embeddings.npz")["heldout_emb"][0]
    o = OracleEnvs(cfg, 2, seed=21, task_embedding=task)
    o.reset()
    for t in range(30):
        o.step(o.scripted_actions(t))
    return o, task


def test_obs_tile_window(rollout):
    o, _ = rollout
    d = layout.unflatten(o.obs)
    st = split_state(o.get_state(), o.n_envs, o.S, o.P)
    tile = d["Tile"]
    for e in range(o.n_envs):
        for p in range(o.P):
            if not o.mask[e, p] or not st["ent"][e, abi.F["alive"], p]:
                continue
            r, c = st["ent"][e, abi.F["row"], p], st["ent"][e, abi.F["col"], p]
            # centre row 112 is the agent's own tile, absolute coords (baseline_policy.py:96-104)
            assert tuple(tile[e, p, 112, :2]) == (r, c)
            assert tile[e, p, :, 2].max() <= 15 and tile[e, p, :, 2].min() >= 0
            win = st["mat"][e, r - 7:r + 8, c - 7:c + 8].reshape(-1)
            assert np.array_equal(tile[e, p, :, 2], win)


def test_obs_entity_and_masks(rollout):
    o, _ = rollout
    d = layout.unflatten(o.obs)
    ent, at = d["Entity"], d["ActionTargets"]
    found = 0
    for e in range(o.n_envs):
        for p in range(o.P):
            if not np.any(o.obs[e, p]):
                continue
            ids = ent[e, p, :, 0]
            my = d["AgentId"][e, p, 0]
            assert 1 <= my <= 128 and my in ids  # own row found by id match (baseline_policy.py:132-140)
            assert set(np.unique(ent[e, p, :, 1])) <= {0, 1, 2, 3}  # npc_type
            n = int((ids != 0).sum())
            assert np.all(ids[n:] == 0)
            tgt = at["Attack"]["Target"][e, p]
            assert tgt.shape == (101,) and tgt[100] == 1  # noop is the last index
            me = np.where(ids == my)[0][0]
            for i in np.where(tgt[:100] == 1)[0]:  # mask[i] <-> Entity row i (yaofeng/reward_wrapper.py:79-80)
                assert ids[i] != 0 and ids[i] != my
                dr = abs(ent[e, p, i, 2] - ent[e, p, me, 2])
                dc = abs(ent[e, p, i, 3] - ent[e, p, me, 3])
                assert max(dr, dc) <= 3
                found += 1
            for (a, b) in [("Destroy", "InventoryItem"), ("Give", "InventoryItem"),
                           ("Sell", "InventoryItem"), ("Use", "InventoryItem")]:
                m = at[a][b][e, p]
                assert m.shape == (13,) and m[-1] == 1  # yaofeng/reward_wrapper.py:71-75
            assert at["Buy"]["MarketItem"][e, p][-1] == 1
            assert at["Move"]["Direction"][e, p].shape == (5,)
            assert at["Move"]["Direction"][e, p][4] == 1  # Stay on a habitable tile
    assert found > 0


def test_obs_task_is_heldout_embedding(rollout):
    o, task = rollout
    d = layout.unflatten(o.obs)
    alive = o.obs.reshape(-1, o.obs_elems).any(1).reshape(o.n_envs, o.P)
    assert np.array_equal(d["Task"][alive], np.broadcast_to(task.astype(np.float32), d["Task"][alive].shape))


def test_ids_and_materials(rollout):
    o, _ = rollout
    st = split_state(o.get_state(), o.n_envs, o.S, o.P)
    ids = st["ent"][:, abi.F["id"]]
    assert np.array_equal(ids[:, :128], np.tile(np.arange(1, 129), (o.n_envs, 1)))  # train_helper.py:147
    npc = ids[:, 128:]
    alive_npc = st["ent"][:, abi.F["alive"], 128:] == 1
    assert np.all(npc[alive_npc] < 0)  # NPC ids are negative (stat_wrapper.py:284-285)
    bank = o.map_bank()
    assert bank.shape == (4, 160, 160) and bank.max() <= 15  # MAP_CENTER 128 + border
    assert np.all(bank[:, :16, :] == 0) and np.all(bank[:, 144:, :] == 0)


def test_unpack_batched_obs_serves_the_reference_policy_reads():
    """layout.unpack_batched_obs(flat, driver_env.unflatten_context) -- the reference's call at
    baseline_policy.py:41 -- yields what encode_observations / ActionDecoder index (:42-76,
    :230-262), as views of the flat batch (the start-kit's in-place Tile edit lands in it)."""
    import torch

    from nmmo_amd.layout import ACTION_HEADS, flat_layout, unpack_batched_obs

    ctx = flat_layout(2048)
    flat = torch.arange(3 * 23987, dtype=torch.float32).reshape(3, 23987)
    d = unpack_batched_obs(flat, ctx)
    assert d["Tile"].shape == (3, 225, 3) and d["Entity"].shape == (3, 100, 31)
    assert d["AgentId"][:, 0].shape == (3,) and d["Inventory"].shape == (3, 12, 16)
    assert d["Market"].shape == (3, 1024, 16) and d["Task"].shape == (3, 2048)
    for (a, b), n in ACTION_HEADS:
        assert d["ActionTargets"][a][b].shape == (3, n)
    d["Tile"][:, :, :2] += 7  # baseline_policy.py:97, on the views
    assert float(flat[0, ctx["Tile"].offset]) == ctx["Tile"].offset + 7
    with pytest.raises(ValueError):
        unpack_batched_obs(flat[:, :-1], ctx)
