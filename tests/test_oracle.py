"""Known-answer tests of the CPU oracle against SPEC.md, one rule per test, on hand-built states
(numbers computed by hand from the SPEC constants, not from the oracle). CPU only."""

import numpy as np
import pytest

from nmmo_amd import abi
from nmmo_amd.config import Config
from oracle.oracle import OracleEnvs, join_state, split_state

F, E = abi.F, abi.E
FOILAGE, WATER, GRASS, SCRUB, STONE = 4, 1, 2, 3, 5


def make(systems, P=4, seed=3):
    cfg = Config(systems=systems, PLAYER_N=P, MAP_N=1, early_stop_agent_num=0)
    o = OracleEnvs(cfg, 1, seed=seed)
    o.reset()
    return o, split_state(o.get_state(), 1, o.S, o.P)


def put(o, d):
    o.set_state(join_state(d))


NOOP = [0, 100, 1024, 12, 12, 100, 0, 100, 4, 12, 0, 12]  # last index of every target/item head


def noop_actions(o):
    return np.tile(np.array(NOOP, np.int32), (1, o.P, 1))


def find_tile(mat, pred, avoid=()):
    for r in range(24, 136):
        for c in range(24, 136):
            if (r, c) not in avoid and pred(mat, r, c):
                return r, c
    raise AssertionError("no such tile")


def nbrs(mat, r, c):
    return [mat[r - 1, c], mat[r + 1, c], mat[r, c - 1], mat[r, c + 1]]


def plain(mat, r, c):  # grass, no water around, not foilage
    return mat[r, c] == GRASS and WATER not in nbrs(mat, r, c)


def place(d, slot, r, c, **fields):
    d["ent"][0, F["row"], slot] = r
    d["ent"][0, F["col"], slot] = c
    for k, v in fields.items():
        d["ent"][0, F[k], slot] = v


def park_others(d, keep, mat):
    """Move players not in `keep` to distinct plain tiles far from the scenario."""
    spots = [(r, c) for r in range(120, 140) for c in range(120, 140) if plain(mat, r, c)]
    k = 0
    for s in range(d["ent"].shape[2]):
        if s in keep or d["ent"][0, F["alive"], s] == 0 or d["ent"][0, F["id"], s] <= 0:
            continue
        place(d, s, *spots[k])
        k += 1


def visible_index(d, p, target):
    ent = d["ent"][0]
    r, c = ent[F["row"], p], ent[F["col"], p]
    rows = sorted((ent[F["ds_row"], s], s) for s in range(ent.shape[1])
                  if ent[F["alive"], s] and max(abs(ent[F["row"], s] - r), abs(ent[F["col"], s] - c)) <= 7)
    return [s for _, s in rows].index(target)


def test_starvation_and_dehydration():
    o, d = make(("Resource",))
    mat = d["mat"][0]
    r, c = find_tile(mat, plain)
    park_others(d, {0}, mat)
    place(d, 0, r, c, food=0, water=0, health=50, resilient=0)
    place(d, 1, *find_tile(mat, plain, avoid=[(r, c)] + [(x, y) for x in range(120, 140) for y in range(120, 140)]),
          food=0, water=0, health=50, resilient=1)
    put(o, d)
    o.step(noop_actions(o))
    s = split_state(o.get_state(), 1, o.S, o.P)["ent"][0]
    assert s[F["health"], 0] == 30 and s[F["health_restore"], 0] == -20  # 10 + 10
    assert s[F["health"], 1] == 40  # resilient: int(10 * 0.5) each
    assert s[F["food"], 0] == 0 and s[F["water"], 0] == 0


def test_regen_and_depletion():
    o, d = make(("Resource",))
    mat = d["mat"][0]
    park_others(d, {0}, mat)
    place(d, 0, *find_tile(mat, plain), food=60, water=60, health=50)
    put(o, d)
    o.step(noop_actions(o))
    s = split_state(o.get_state(), 1, o.S, o.P)["ent"][0]
    assert (s[F["health"], 0], s[F["food"], 0], s[F["water"], 0]) == (60, 55, 55)


def test_first_player_on_foilage_eats():
    o, d = make(("Resource",))
    mat = d["mat"][0]
    r, c = find_tile(mat, lambda m, r, c: m[r, c] == FOILAGE and WATER not in nbrs(m, r, c))
    park_others(d, {0, 1}, mat)
    place(d, 0, r, c, food=40, water=40)
    place(d, 1, r, c, food=40, water=40)
    put(o, d)
    o.step(noop_actions(o))
    s = split_state(o.get_state(), 1, o.S, o.P)
    assert s["ent"][0][F["food"], 0] == 100  # slot 0 harvests
    assert s["ent"][0][F["food"], 1] == 35   # slot 1 sees Scrub
    assert s["mat"][0][r, c] in (SCRUB, FOILAGE)  # Scrub unless the 2.5 % respawn fired


def test_drink_adjacent_water():
    o, d = make(("Resource",))
    mat = d["mat"][0]
    park_others(d, {0}, mat)
    place(d, 0, *find_tile(mat, lambda m, r, c: m[r, c] == GRASS and WATER in nbrs(m, r, c)), water=10)
    put(o, d)
    o.step(noop_actions(o))
    assert split_state(o.get_state(), 1, o.S, o.P)["ent"][0][F["water"], 0] == 100


COMBAT = ("Resource", "Combat", "Progression")


def duel(dist=2, t_fields=None, style=0, both_attack=False, x_fields=None):
    o, d = make(COMBAT)
    mat = d["mat"][0]
    r, c = find_tile(mat, lambda m, r, c: all(plain(m, r, c + k) for k in range(0, 5)))
    park_others(d, {0, 1}, mat)
    place(d, 0, r, c, **{"time_alive": 50, **(x_fields or {})})
    place(d, 1, r, c + dist, **{"time_alive": 50, **(t_fields or {})})
    put(o, d)
    a = noop_actions(o)
    a[0, 0, 0], a[0, 0, 1] = style, visible_index(d, 0, 1)
    if both_attack:
        a[0, 1, 0], a[0, 1, 1] = 0, visible_index(d, 1, 0)
    o.step(a)
    return o, split_state(o.get_state(), 1, o.S, o.P)


def test_melee_damage_equal_skills():
    o, s = duel()
    ent = s["ent"][0]
    # offense 10+5*1 = 15, defense 5*1 = 5, mult 1.0 -> 10
    assert ent[F["health"], 1] == 90 and ent[F["damage"], 1] == 10 and ent[F["attacker_id"], 1] == 1
    assert ent[F["melee_exp"], 0] == 6 and ent[F["melee_level"], 0] == 1
    tick = s["env"][0, E["tick"]]
    assert ent[F["latest_combat_tick"], 0] == tick and ent[F["latest_combat_tick"], 1] == tick


def test_weakness_multiplier():
    # target dominant skill = range (exp 90 -> level 2): melee beats range -> 1.5*15 - 10 = 12.5 -> 12
    _, s = duel(t_fields=dict(range_exp=90, range_level=2))
    assert s["ent"][0][F["health"], 1] == 88
    # mage is not range's weakness: max(15 - 10, 3.75) -> 5
    _, s = duel(t_fields=dict(range_exp=90, range_level=2), style=2)
    assert s["ent"][0][F["health"], 1] == 95


def test_minimum_damage_proportion():
    lv = {f"{k}_level": 10 for k in ["melee", "range", "mage", "fishing", "herbalism",
                                       "prospecting", "carving", "alchemy"]}
    _, s = duel(t_fields=lv)  # defense 50 -> int(0.25 * 15) = 3
    assert s["ent"][0][F["health"], 1] == 97


def test_spawn_immunity_and_reach():
    _, s = duel(t_fields=dict(time_alive=5))  # 6 after the update, < 20
    assert s["ent"][0][F["health"], 1] == 100 and s["ent"][0][F["melee_exp"], 0] == 0
    _, s = duel(dist=4)
    assert s["ent"][0][F["health"], 1] == 100


def test_kill_cull_and_serial_order():
    # slot 0 acts first and kills slot 1 (health 5, no regen at food/water 40) -> slot 1's
    # counter-attack never executes (Realm.step serial order)
    o, s = duel(t_fields=dict(health=5, food=40, water=40), both_attack=True,
                x_fields=dict(food=40, water=40, health=70))
    ent, env = s["ent"][0], s["env"][0]
    assert ent[F["alive"], 1] == 0 and ent[F["died_tick"], 1] == env[E["tick"]]
    assert ent[F["health"], 0] == 70 and ent[F["player_kills"], 0] == 1
    assert o.term[0, 1] == 1 and o.rew[0, 1] == -1.0 and o.mask[0, 1] == 1
    assert o.rew[0, 0] == np.float32(1 / 1024)
    assert env[E["players_alive"]] == o.P - 1
    ring = s["ring"][0]
    assert ring[(env[E["free_head"]] + env[E["free_count"]] - 1) % o.S] == ent[F["ds_row"], 1]


def test_move_blocked_by_stone():
    o, d = make(("Resource",))
    mat = d["mat"][0]
    passable = (GRASS, SCRUB, FOILAGE)
    r, c = find_tile(mat, lambda m, r, c: m[r, c] in passable and m[r - 1, c] == STONE
                     and m[r + 1, c] in passable)
    park_others(d, {0}, mat)
    place(d, 0, r, c)
    put(o, d)
    a = noop_actions(o)
    a[0, 0, 8] = 0  # North into stone
    o.step(a)
    ent = split_state(o.get_state(), 1, o.S, o.P)["ent"][0]
    assert (ent[F["row"], 0], ent[F["col"], 0]) == (r, c)
    a[0, 0, 8] = 1  # South onto grass
    o.step(a)
    ent = split_state(o.get_state(), 1, o.S, o.P)["ent"][0]
    assert (ent[F["row"], 0], ent[F["col"], 0]) == (r + 1, c)


def test_horizon_truncation_then_auto_reset():
    o, d = make(("Resource",))
    d["env"][0, E["tick"]] = 1023
    put(o, d)
    o.step(noop_actions(o))
    env = split_state(o.get_state(), 1, o.S, o.P)["env"][0]
    assert env[E["done"]] == 1 and env[E["tick"]] == 1024
    assert o.trunc[0].sum() == o.P
    o.step(noop_actions(o))  # pufferlib auto-reset
    env = split_state(o.get_state(), 1, o.S, o.P)["env"][0]
    assert env[E["tick"]] == 0 and env[E["episode"]] == 1 and env[E["done"]] == 0
    assert o.mask[0].sum() == o.P and o.rew[0].sum() == 0


def test_npc_bookkeeping_invariants():
    cfg = Config.preset("C3", MAP_N=2, early_stop_agent_num=8)
    o = OracleEnvs(cfg, 3, seed=9)
    o.reset()
    for t in range(80):
        o.step(o.scripted_actions(t))
        s = split_state(o.get_state(), 3, o.S, o.P)
        for e in range(3):
            ent, env, ring = s["ent"][e], s["env"][e], s["ring"][e]
            alive = ent[F["alive"]] == 1
            n_npc = env[E["npc_count"]]
            assert 0 <= n_npc <= 256
            assert np.all(alive[128:128 + n_npc]) and not np.any(alive[128 + n_npc:])  # compacted
            ids = ent[F["id"], 128:128 + n_npc]
            assert np.all(np.diff(ids) < 0)  # spawn order = decreasing ids
            rows = list(ent[F["ds_row"]][alive])
            fr = [ring[(env[E["free_head"]] + k) % o.S] for k in range(env[E["free_count"]])]
            assert sorted(rows + fr) == list(range(1, o.S + 1))  # every datastore row exactly once
            assert env[E["players_alive"]] == alive[:128].sum()


def test_determinism_and_seed_sensitivity():
    cfg = Config.preset("C3", MAP_N=2)
    runs = []
    for seed in (4, 4, 5):
        o = OracleEnvs(cfg, 2, seed=seed)
        o.reset()
        for t in range(25):
            o.step(o.scripted_actions(t))
        runs.append(o.get_state())
    assert np.array_equal(runs[0], runs[1]) and not np.array_equal(runs[0], runs[2])


@pytest.mark.parametrize("preset", ["C2", "C3"])
def test_golden_rollout_hashes(preset):
    """Regression pin: the committed hashes were produced by tests/golden/make_rollout_fixtures.py
    (self-generated from the oracle — parity vs nmmo 2.1 is unpinned, SPEC.md)."""
    import json

    from tests.golden.make_rollout_fixtures import rollout_hashes

    golden = json.load(open("tests/golden/rollout_hashes.json"))[preset]
    assert rollout_hashes(preset) == golden


# ---------------------------------------------------------------- items (SPEC §9)
ITEMS = ("Resource", "Combat", "Progression", "Item", "Equipment", "Profession", "Exchange")
ORE, SLAG = 7, 6


def item_words(typ, level=1, qty=1, row=1, equipped=0, price=0, ltick=0):
    return [typ | (level << 5) | (equipped << 9) | (price << 10) | (ltick << 17), qty | (row << 16)]


def give_item(d, p, k, words):
    d["items"][0, p, k] = words
    # take the row out of the free ring (rows 1..12P start in order; use the last ones)


def test_harvest_ore_without_tool():
    o, d = make(ITEMS)
    mat = d["mat"][0]
    r, c = find_tile(mat, lambda m, r, c: m[r, c] in (GRASS, SCRUB) and WATER not in nbrs(m, r, c))
    d["mat"][0][r, c] = ORE
    park_others(d, {0}, mat)
    place(d, 0, r, c)
    put(o, d)
    o.step(noop_actions(o))
    s = split_state(o.get_state(), 1, o.S, o.P)
    it = s["items"][0, 0, 0]
    assert (it[0] & 31, (it[0] >> 5) & 15, it[1] & 0xFFFF) == (13, 1, 1)  # Whetstone L1 x1
    assert it[1] >> 16 == 1  # first row of the FIFO ring
    assert s["ent"][0][F["prospecting_exp"], 0] == 15
    assert s["mat"][0][r, c] in (SLAG, ORE)  # depleted (unless the 10 % respawn fired)
    assert s["env"][0, E["item_free_count"]] == 12 * o.P - 1


def _with_item(words, slot=0, **fields):
    o, d = make(ITEMS)
    mat = d["mat"][0]
    park_others(d, {0}, mat)
    place(d, 0, *find_tile(mat, plain), **fields)
    row = words[1] >> 16
    d["items"][0, 0, slot] = words
    ring = d["iring"][0]
    # remove `row` from the free ring: rows are 1..12P in order, head 0
    keep = [x for x in ring if x != row]
    d["iring"][0] = keep + [0]
    d["env"][0, E["item_free_count"]] -= 1
    put(o, d)
    return o, d


def test_use_ration_restores_food_and_water():
    o, d = _with_item(item_words(16, level=1, row=7), food=20, water=30, health=100)
    a = noop_actions(o)
    a[0, 0, 11] = 0  # Use.InventoryItem 0
    o.step(a)
    s = split_state(o.get_state(), 1, o.S, o.P)
    # update first: 20-5, 30-5; then +55 each (50 + 5*1)
    assert (s["ent"][0][F["food"], 0], s["ent"][0][F["water"], 0]) == (70, 80)
    assert s["items"][0, 0, 0, 0] == 0  # consumed
    ring, env = s["iring"][0], s["env"][0]
    assert ring[(env[E["item_free_head"]] + env[E["item_free_count"]] - 1) % (12 * o.P)] == 7


def test_equip_weapon_adds_offense():
    o, d = _with_item(item_words(5, level=1, row=3), time_alive=50)  # Spear L1: +10 melee attack
    a = noop_actions(o)
    a[0, 0, 11] = 0
    o.step(a)
    s = split_state(o.get_state(), 1, o.S, o.P)
    assert (s["items"][0, 0, 0, 0] >> 9) & 1 == 1 and s["ent"][0][F["item_level"], 0] == 1
    # now attack a player 2 tiles away: offense 15 + 10 = 25, defense 5 -> 20
    d = split_state(o.get_state(), 1, o.S, o.P)
    r, c = d["ent"][0][F["row"], 0], d["ent"][0][F["col"], 0]
    place(d, 1, r, c + 2, time_alive=50)
    put(o, d)
    a = noop_actions(o)
    a[0, 0, 0], a[0, 0, 1] = 0, visible_index(d, 0, 1)
    o.step(a)
    s = split_state(o.get_state(), 1, o.S, o.P)
    assert s["ent"][0][F["damage"], 1] == 20


def test_sell_then_buy_moves_gold_and_item():
    o, d = _with_item(item_words(2, level=1, row=9), gold=0)  # a Hat
    d = split_state(o.get_state(), 1, o.S, o.P)
    r, c = d["ent"][0][F["row"], 0], d["ent"][0][F["col"], 0]
    place(d, 1, r, c + 1, gold=50)
    put(o, d)
    a = noop_actions(o)
    a[0, 0, 9], a[0, 0, 10] = 0, 9  # Sell item 0 at price 10
    o.step(a)
    s = split_state(o.get_state(), 1, o.S, o.P)
    assert (s["items"][0, 0, 0, 0] >> 10) & 127 == 10
    a = noop_actions(o)
    a[0, 1, 2] = 0  # Buy market listing 0
    o.step(a)
    s = split_state(o.get_state(), 1, o.S, o.P)
    assert s["ent"][0][F["gold"], 0] == 10 and s["ent"][0][F["gold"], 1] == 40
    assert s["items"][0, 0, 0, 0] == 0 and (s["items"][0, 1, 0, 0] & 31) == 2
    assert (s["items"][0, 1, 0, 0] >> 10) & 127 == 0 and s["items"][0, 1, 0, 1] >> 16 == 9


def test_give_requires_same_tile():
    for dist, moved in [(0, True), (1, False)]:
        o, d = _with_item(item_words(17, level=1, row=5))
        d = split_state(o.get_state(), 1, o.S, o.P)
        r, c = d["ent"][0][F["row"], 0], d["ent"][0][F["col"], 0]
        place(d, 1, r, c + dist)
        put(o, d)
        a = noop_actions(o)
        a[0, 0, 4], a[0, 0, 5] = 0, visible_index(d, 0, 1)  # Give item 0 to player 2
        o.step(a)
        s = split_state(o.get_state(), 1, o.S, o.P)
        assert ((s["items"][0, 1, 0, 0] & 31) == 17) == moved


# ---------------------------------------------------------------- event log (SPEC §11)
EV = abi.EventCode
C = abi.ATTR_TO_COL


def test_event_log_eat_and_drink():
    o, d = make(("Resource",))
    mat = d["mat"][0]
    r, c = find_tile(mat, lambda m, r, c: m[r, c] in (GRASS, SCRUB) and WATER in nbrs(m, r, c))
    d["mat"][0][r, c] = FOILAGE
    park_others(d, {0}, mat)
    place(d, 0, r, c)
    put(o, d)
    a = noop_actions(o)
    o.step(a)
    ev = o.events(0)
    mine = ev[ev[:, C["ent_id"]] == 1]
    # update phase (eat, drink), then Move (Stay still sets the first exploration record)
    assert [tuple(x) for x in mine[:, [C["event"], C["tick"]]]] == [
        (EV.EAT_FOOD, 1), (EV.DRINK_WATER, 1), (EV.GO_FARTHEST, 1)]
    assert mine[2, C["distance"]] == 64 - max(abs(r - 80), abs(c - 80))
    assert np.array_equal(ev[:, C["id"]], np.arange(1, len(ev) + 1))  # running ids
    assert split_state(o.get_state(), 1, o.S, o.P)["env"][0, E["event_count"]] == len(ev)


def test_event_log_hit_kill_and_cull():
    o, s = duel(t_fields=dict(health=5, food=40, water=40), x_fields=dict(food=40, water=40))
    ev = o.events(0)
    codes = [int(x) for x in ev[:, C["event"]]]
    hit = ev[ev[:, C["event"]] == EV.SCORE_HIT][0]
    assert hit[C["ent_id"]] == 1 and hit[C["combat_style"]] == 1 and hit[C["damage"]] == 10
    kill = ev[ev[:, C["event"]] == EV.PLAYER_KILL][0]
    assert kill[C["ent_id"]] == 1 and kill[C["target_ent"]] == 2 and kill[C["level"]] == 1
    culled = ev[ev[:, C["event"]] == EV.AGENT_CULLED]
    assert culled[:, C["ent_id"]].tolist() == [2]
    # phase order: attack events, then the cull
    assert codes.index(EV.SCORE_HIT) < codes.index(EV.PLAYER_KILL) < codes.index(EV.AGENT_CULLED)


def test_event_log_ring_keeps_latest_rows():
    cfg = Config.preset("C2", MAP_N=1, early_stop_agent_num=0, event_cap=16)
    o = OracleEnvs(cfg, 1, seed=4)
    o.reset()
    for t in range(6):
        o.step(o.scripted_actions(t))
    n = split_state(o.get_state(), 1, o.S, o.P)["env"][0, E["event_count"]]
    assert n > 16
    ev = o.events(0)
    assert len(ev) == 16 and ev[-1, C["id"]] == n and np.all(np.diff(ev[:, C["id"]]) == 1)
    off = OracleEnvs(Config.preset("C2", MAP_N=1, event_cap=0), 1, seed=4)
    off.reset()
    off.step(off.scripted_actions(0))
    assert len(off.events(0)) == 0
    assert split_state(off.get_state(), 1, off.S, off.P)["env"][0, E["event_count"]] == 0


def test_event_log_harvest_item():
    o, d = make(ITEMS)
    mat = d["mat"][0]
    r, c = find_tile(mat, lambda m, r, c: m[r, c] in (GRASS, SCRUB) and WATER not in nbrs(m, r, c))
    d["mat"][0][r, c] = ORE
    park_others(d, {0}, mat)
    place(d, 0, r, c)
    put(o, d)
    o.step(noop_actions(o))
    ev = o.events(0)
    h = ev[(ev[:, C["event"]] == EV.HARVEST_ITEM) & (ev[:, C["ent_id"]] == 1)]
    assert h.shape[0] == 1 and (h[0, C["item_type"]], h[0, C["level"]], h[0, C["quantity"]]) == (13, 1, 1)


def _npc_scenario(wall):
    """A hostile NPC 3 tiles west of player 1 on open grass; `wall` = list of (dr, dc) offsets
    from the NPC that are turned to Stone. Returns (o, npc_slot, (r, c))."""
    o, d = make(("Resource", "Combat", "NPC"), P=4)
    mat = d["mat"][0]
    r, c = 60, 60
    mat[r - 8:r + 9, c - 8:c + 12] = GRASS  # an open field (tiles off the bank material never respawn: grass)
    park_others(d, {0}, mat)
    place(d, 0, r, c + 3)
    ent = d["ent"][0]
    n = o.P  # first NPC slot; move every other NPC far away
    for s in range(o.P + 1, o.S):
        if ent[F["alive"], s]:
            place(d, s, 30 + (s % 50), 30 + (s // 50))
    place(d, n, r, c, npc_type=3, target_id=1, attacker_id=0, health=100)
    for dr, dc in wall:
        mat[r + dr, c + dc] = STONE
    put(o, d)
    return o, n, (r, c)


def test_npc_hunt_takes_shortest_path_around_a_wall():
    """SPEC §6 v2: BFS inside the 15x15 window. A wall at column +1 (rows -2..+2) between the NPC
    and its target: both N and S start a shortest path around it; N comes first. (The v1 greedy
    rule would try E, find Stone, and stay because the row offset is 0.)"""
    o, n, (r, c) = _npc_scenario([(i, 1) for i in range(-2, 3)])
    o.step(noop_actions(o))
    ent = split_state(o.get_state(), 1, o.S, o.P)["ent"][0]
    assert (ent[F["row"], n], ent[F["col"], n]) == (r - 1, c)


def test_npc_hunt_prefers_first_direction_on_open_ground():
    """No obstacle: N/S/E/W order among the shortest-path first steps; target due east -> E."""
    o, n, (r, c) = _npc_scenario([])
    o.step(noop_actions(o))
    ent = split_state(o.get_state(), 1, o.S, o.P)["ent"][0]
    assert (ent[F["row"], n], ent[F["col"], n]) == (r, c + 1)


def test_npc_hunt_unreachable_falls_back_to_greedy():
    """Target walled in on all sides inside the window: the v1 greedy step (E is Stone, row offset
    0) -> stay."""
    ring = [(i, j) for i in range(-1, 2) for j in range(2, 5) if (i, j) != (0, 3)]
    o, n, (r, c) = _npc_scenario(ring)
    o.step(noop_actions(o))
    ent = split_state(o.get_state(), 1, o.S, o.P)["ent"][0]
    assert (ent[F["row"], n], ent[F["col"], n]) == (r, c + 1)  # E is open here: greedy steps E
