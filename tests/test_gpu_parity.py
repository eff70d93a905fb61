"""HIP path vs the CPU oracle, bit-exact (SPEC.md v1). Calls go through the C-ABI
(libnmmo_hip.so via nmmo_amd.engine); the oracle is only the checker."""

import numpy as np
import pytest

from nmmo_amd import abi
from nmmo_amd.config import Config
from oracle.oracle import OracleEnvs, join_state, split_state

pytestmark = pytest.mark.gpu


def _engine(cfg, n_envs, seed, task=None):
    import torch

    from nmmo_amd.engine import NmmoEngine

    assert torch.cuda.is_available()
    return NmmoEngine(cfg, n_envs, seed=seed, task_embedding=task)


def _cmp_state(ga, oa, n, S, where, P=128):
    g = split_state(ga, n, S, P)
    o = split_state(oa, n, S, P)
    g["tstate"], o["tstate"] = g["tstate"].view(np.uint8), o["tstate"].view(np.uint8)
    for key in ("env", "ring", "mat", "items", "iring", "tasks", "tstate"):
        if not np.array_equal(g[key], o[key]):
            bad = np.argwhere(g[key] != o[key])[:5]
            raise AssertionError(f"{where}: {key} differs at {bad.tolist()}")
    if not np.array_equal(g["ent"], o["ent"]):
        bad = np.argwhere(g["ent"] != o["ent"])[:8]
        names = [(int(e), abi.ENTITY_FIELDS[f] if f < len(abi.ENTITY_FIELDS) else f, int(s),
                  int(g["ent"][e, f, s]), int(o["ent"][e, f, s])) for e, f, s in bad]
        raise AssertionError(f"{where}: entity fields differ (env, field, slot, gpu, oracle): {names}")


def _cmp_events(eng, orc, n, where):
    for e in range(n):
        g, o = eng.events(e), orc.events(e)
        if g.shape != o.shape or not np.array_equal(g, o):
            k = next((i for i in range(min(len(g), len(o))) if not np.array_equal(g[i], o[i])), None)
            raise AssertionError(f"{where}: env {e} event log differs (gpu {len(g)} rows, oracle "
                                 f"{len(o)}); first differing row {k}: gpu {g[k].tolist() if k is not None else None} "
                                 f"oracle {o[k].tolist() if k is not None else None}")


def test_map_bank_parity():
    cfg = Config.preset("C2", MAP_N=16, map_seed=123)
    eng = _engine(cfg, 1, seed=0)
    orc = OracleEnvs(cfg, 1, seed=0)
    assert np.array_equal(eng.map_bank(), orc.map_bank())


@pytest.mark.parametrize("preset", ["C2", "C3", "C4"])
def test_rollout_parity(preset):
    import torch

    n, steps = 6, 120
    task = (np.arange(2048) % 97 / 97.0 - 0.5).astype(np.float16)
    cfg = Config.preset(preset, MAP_N=8, early_stop_agent_num=8)
    eng = _engine(cfg, n, seed=11, task=task)
    orc = OracleEnvs(cfg, n, seed=11, task_embedding=task)
    eng.reset()
    orc.reset()
    torch.cuda.synchronize()
    _cmp_state(eng.get_state(), orc.get_state(), n, eng.S, "reset")
    if orc.obs is not None:
        assert np.array_equal(eng.obs.cpu().numpy(), orc.obs), "reset obs"
    assert np.array_equal(eng.mask.cpu().numpy(), orc.mask)
    for t in range(steps):
        acts = orc.scripted_actions(1000 + t)
        g_acts = eng.scripted_actions(1000 + t)
        assert np.array_equal(g_acts.cpu().numpy(), acts), f"policy differs at step {t}"
        orc.step(acts)
        eng.step(torch.from_numpy(acts).cuda())
        torch.cuda.synchronize()
        _cmp_state(eng.get_state(), orc.get_state(), n, eng.S, f"step {t}")
        for name in ("rew", "term", "trunc", "mask"):
            gv = getattr(eng, name).cpu().numpy()
            ov = getattr(orc, name)
            assert np.array_equal(gv, ov), f"{name} differs at step {t}"
        _cmp_events(eng, orc, n, f"step {t}")
        if orc.obs is not None and (t % 10 == 0 or t == steps - 1):
            go = eng.obs.cpu().numpy()
            if not np.array_equal(go, orc.obs):
                bad = np.argwhere(go != orc.obs)[:5]
                raise AssertionError(f"obs differs at step {t}: {bad.tolist()}")


def test_set_state_roundtrip():
    import torch

    cfg = Config.preset("C3", MAP_N=4)
    orc = OracleEnvs(cfg, 3, seed=5)
    orc.reset()
    for t in range(15):
        orc.step(orc.scripted_actions(t))
    eng = _engine(cfg, 3, seed=99)
    eng.set_state(orc.get_state())
    for t in range(15, 40):
        a = orc.scripted_actions(t)
        orc.step(a)
        eng.step(torch.from_numpy(a).cuda())
    torch.cuda.synchronize()
    _cmp_state(eng.get_state(), orc.get_state(), 3, eng.S, "after set_state")


def test_foreign_depletion_parity():
    """Without professions the tick's respawn assumes every depleted tile is eaten Foilage and
    skips the map-bank read (tick.hip, DevState::foreign). A set_state that depletes Tree and Ore
    tiles instead must switch it back to the bank: the restored materials and their respawn
    probabilities then differ from Foilage's, so any shortcut shows up in `mat`."""
    import torch

    cfg = Config.preset("C2", MAP_N=4)
    n = 3
    orc = OracleEnvs(cfg, n, seed=21)
    orc.reset()
    for t in range(5):
        orc.step(orc.scripted_actions(t))
    d = split_state(orc.get_state(), n, orc.S, 128)
    bank = orc.map_bank().reshape(-1, abi.MAP_SIZE, abi.MAP_SIZE)
    M = {"stump": 8, "tree": 9, "slag": 6, "ore": 7}  # common.h material enum
    changed = 0
    for e in range(n):
        b = bank[d["env"][e, abi.E["map_id"]]]
        for src, dst in (("tree", "stump"), ("ore", "slag")):
            rr, cc = np.nonzero((b == M[src]) & (d["mat"][e] == M[src]))
            d["mat"][e, rr[:40], cc[:40]] = M[dst]
            changed += min(40, rr.size)
    assert changed > 40
    orc.set_state(join_state(d))
    eng = _engine(cfg, n, seed=21)
    eng.set_state(orc.get_state())
    for t in range(5, 45):
        a = orc.scripted_actions(t)
        orc.step(a)
        eng.step(torch.from_numpy(a).cuda())
        torch.cuda.synchronize()
        _cmp_state(eng.get_state(), orc.get_state(), n, eng.S, f"step {t}")
        if t == 25:  # most of the stumps have grown back into trees (p = 0.1 per tick)
            m = split_state(orc.get_state(), n, orc.S, 128)["mat"]
            assert sum(int(((m[e] == M["tree"]) & (d["mat"][e] == M["stump"])).sum()) for e in range(n)) > 60


def test_set_state_rejects_changed_slim_fields():
    """Without Item/Equipment/Profession/Exchange (C3) the tick keeps 15 entity fields in HBM as
    reset wrote them (tick.hip slim table); a blob that changes one of them is refused."""
    from nmmo_amd._native import NativeError

    cfg = Config.preset("C3", MAP_N=4)
    eng = _engine(cfg, 2, seed=3)
    eng.reset()
    blob = eng.get_state()
    eng.set_state(blob)  # a state the engine produced is accepted
    st = split_state(blob.copy(), 2, eng.S, 128)
    per = blob.nbytes // 2
    off = 16 * 4 + (abi.ENTITY_FIELDS.index("gold") * eng.S + 5) * 2  # env 0, player slot 5, gold
    bad = blob.copy()
    bad[off:off + 2] = np.array([7], np.int16).view(np.uint8)
    assert split_state(bad, 2, eng.S, 128)["ent"][0, abi.ENTITY_FIELDS.index("gold"), 5] == 7
    assert st["ent"].shape[1] >= 45 and per > off
    with pytest.raises(NativeError):
        eng.set_state(bad)


class _EngineStepper:
    """HIP engine behind the golden-rollout driver (numpy in/out)."""

    def __init__(self, preset):
        from tests.golden.make_rollout_fixtures import config

        self.e = _engine(config(preset), 4, seed=2024)

    def reset(self):
        self.e.reset()

    def step(self, a):
        import torch

        self.e.step(torch.from_numpy(a).cuda())

    def scripted_actions(self, s):
        return self.e.scripted_actions(s).cpu().numpy()

    def get_state(self):
        import torch

        torch.cuda.synchronize()
        return self.e.get_state()

    def outputs(self):
        return tuple(getattr(self.e, n).cpu().numpy() for n in ("rew", "term", "trunc", "mask"))

    def events(self, e):
        return self.e.events(e)


@pytest.mark.parametrize("preset", ["C2", "C3"])
def test_golden_rollout_hashes_gpu(preset):
    import json

    from tests.golden.make_rollout_fixtures import rollout

    golden = json.load(open("tests/golden/rollout_hashes.json"))[preset]
    assert rollout(_EngineStepper(preset), preset) == golden


def _stress_items(d, rng, P):
    """Random inventories (rows taken from the front of the item FIFO), equipment, listings,
    gold and same-tile player pairs, so Use/Buy/Give/GiveGold/Destroy/Sell, ammunition and loot
    all fire in the first ticks (SPEC §9)."""
    n = d["env"].shape[0]
    IC = abi.INV_SLOTS * P
    E, F = abi.E, abi.F
    for e in range(n):
        row = 1
        for p in range(P):
            used = set()
            for k in range(int(rng.integers(0, abi.INV_SLOTS + 1))):
                typ = int(rng.integers(2, 18))
                lvl = int(rng.integers(1, 4))
                slot = {2: 0, 3: 1, 4: 2}.get(typ, 3 if 5 <= typ <= 12 else 4 if 13 <= typ <= 15 else -1)
                eq = int(slot >= 0 and slot not in used and rng.random() < 0.4)
                if eq:
                    used.add(slot)
                price = int(rng.integers(1, 40)) if (not eq and rng.random() < 0.3) else 0
                qty = int(rng.integers(1, 4)) if 13 <= typ <= 15 else 1
                d["items"][e, p, k] = [typ | (lvl << 5) | (eq << 9) | (price << 10), qty | (row << 16)]
                row += 1
            d["ent"][e, F["item_level"], p] = sum(
                (int(w0) >> 5) & 15 for w0 in d["items"][e, p, :, 0] if (w0 & 31) and (w0 >> 9) & 1)
        d["iring"][e, :] = 0
        d["iring"][e, :IC - row + 1] = np.arange(row, IC + 1)
        d["env"][e, E["item_free_head"]] = 0
        d["env"][e, E["item_free_count"]] = IC - row + 1
        d["ent"][e, F["gold"], :P] = rng.integers(0, 60, P)
        for p in range(1, P, 2):  # pairs on one tile: Give / GiveGold targets
            d["ent"][e, F["row"], p] = d["ent"][e, F["row"], p - 1]
            d["ent"][e, F["col"], p] = d["ent"][e, F["col"], p - 1]
        d["ent"][e, F["time_alive"], :P] = 30  # past spawn immunity: kills (loot) early


def test_item_stress_parity():
    import torch

    from oracle.oracle import join_state

    n, steps = 4, 60
    cfg = Config.preset("C4", MAP_N=4, early_stop_agent_num=0)
    orc = OracleEnvs(cfg, n, seed=17)
    orc.reset()
    d = split_state(orc.get_state(), n, orc.S, orc.P)
    _stress_items(d, np.random.default_rng(5), orc.P)
    orc.set_state(join_state(d))
    eng = _engine(cfg, n, seed=0)
    eng.set_state(orc.get_state())
    busy = 0
    for t in range(steps):
        acts = orc.scripted_actions(500 + t)
        g_acts = eng.scripted_actions(500 + t)
        if not np.array_equal(g_acts.cpu().numpy(), acts):
            bad = np.argwhere(g_acts.cpu().numpy() != acts)[:5]
            raise AssertionError(f"policy differs at step {t}: {bad.tolist()}")
        busy += int((acts[..., [2, 3, 4, 6, 9, 11]] != [1024, 12, 12, 0, 12, 12]).sum())
        orc.step(acts)
        eng.step(torch.from_numpy(acts).cuda())
        torch.cuda.synchronize()
        _cmp_state(eng.get_state(), orc.get_state(), n, eng.S, f"stress step {t}")
        for name in ("rew", "term", "trunc", "mask"):
            assert np.array_equal(getattr(eng, name).cpu().numpy(), getattr(orc, name)), f"{name} @ {t}"
        _cmp_events(eng, orc, n, f"stress step {t}")
        if t % 5 == 0:
            go = eng.obs.cpu().numpy()
            if not np.array_equal(go, orc.obs):
                bad = np.argwhere(go != orc.obs)[:5]
                raise AssertionError(f"stress obs differs at step {t}: {bad.tolist()}")
    assert busy > 1000  # item heads were actually exercised


def _all_predicate_tasks():
    from nmmo_amd import tasks as T

    return [
        T.task("TickGE", num_tick=40), T.task("CountEvent", event="DRINK_WATER", N=5),
        T.task("CountEvent", event="GO_FARTHEST", N=3), T.task("ScoreHit", combat_style="Melee", N=2),
        T.task("HarvestItem", item="Ration", level=1, quantity=2),
        T.task("ConsumeItem", item="Potion", level=1, quantity=1),
        T.task("ListItem", item="Hat", level=1, quantity=1), T.task("BuyItem", item="Top", level=1, quantity=1),
        T.task("EarnGold", amount=20), T.task("SpendGold", amount=20), T.task("MakeProfit", amount=10),
        T.task("DefeatEntity", agent_type="npc", level=1, num_agent=1),
        T.task("DefeatEntity", agent_type="player", level=1, num_agent=1),
        T.task("HoardGold", amount=50), T.task("AttainSkill", skill="Melee", level=2),
        T.task("GainExperience", skill="Range", experience=30), T.task("EquipItem", item="Spear", level=1),
        T.task("OwnItem", item="Whetstone", level=1, quantity=4), T.task("InventorySpaceGE", space=6),
        T.task("OccupyTile", row=80, col=80), T.task("CanSeeTile", tile_type="Fish"),
        T.task("FullyArmed", combat_style="Melee", level=1),
        T.practice_skill_with_tool("Fishing", 60), T.practice_inventory_management(4, 30),
        T.task("CanSeeAgent", target="left_team_leader"), T.task("CanSeeGroup", target="right_team"),
        T.task("CanSeeAgent", target=5),
    ]


def test_task_parity_all_predicates():
    """Every predicate and both combinators, randomly assigned, on the item-stress scenario:
    rewards and per-player task state (progress, max, accumulators, signals, completion) bit-exact."""
    import torch

    from oracle.oracle import join_state

    n, steps = 4, 50
    cfg = Config.preset("C4", MAP_N=4, early_stop_agent_num=0)
    orc = OracleEnvs(cfg, n, seed=23)
    tl = _all_predicate_tasks()
    rng = np.random.default_rng(9)
    assign = rng.integers(0, len(tl), (n, orc.P)).astype(np.int32)
    emb = rng.standard_normal((len(tl), cfg.TASK_EMBED_DIM)).astype(np.float16)
    orc.set_tasks(tl, emb, assign)
    orc.reset()
    d = split_state(orc.get_state(), n, orc.S, orc.P)
    _stress_items(d, np.random.default_rng(6), orc.P)
    orc.set_state(join_state(d))
    eng = _engine(cfg, n, seed=0)
    eng.set_tasks(tl, emb, assign)
    eng.set_state(orc.get_state())
    for t in range(steps):
        acts = orc.scripted_actions(900 + t)
        orc.step(acts)
        eng.step(torch.from_numpy(acts).cuda())
        torch.cuda.synchronize()
        g, o = split_state(eng.get_state(), n, eng.S, eng.P), split_state(orc.get_state(), n, orc.S, orc.P)
        assert np.array_equal(g["tstate"].view(np.uint8), o["tstate"].view(np.uint8)), f"task state @ {t}"
        _cmp_state(eng.get_state(), orc.get_state(), n, eng.S, f"task step {t}")
        assert np.array_equal(eng.rew.cpu().numpy(), orc.rew), f"rewards @ {t}"
        if t % 10 == 0:
            assert np.array_equal(eng.obs.cpu().numpy(), orc.obs), f"obs @ {t}"
    st = split_state(orc.get_state(), n, orc.S, orc.P)["tstate"]
    assert (st["signals"] > 0).mean() > 0.15 and (st["completed_tick"] > 0).any()


def test_can_see_tile_regrowth_parity_without_npc():
    """CanSeeTile(Foilage) on the Resource-only system set (no NPC spawn barrier): the rewards read
    the tiles the respawn regrows from Scrub in the same tick (tick.hip DevState::tmap barrier).
    Most Foilage starts eaten, so windows gain and lose their Foilage tick to tick."""
    import torch

    from nmmo_amd import tasks as T
    from oracle.oracle import join_state

    n, steps = 4, 60
    cfg = Config.preset("C2", MAP_N=4, early_stop_agent_num=0)
    tl = [T.task("CanSeeTile", tile_type="Foilage"), T.task("TickGE", num_tick=30)]
    assign = np.zeros((n, 128), np.int32)
    assign[:, 1::7] = 1
    orc = OracleEnvs(cfg, n, seed=29)
    orc.set_tasks(tl, None, assign)
    orc.reset()
    d = split_state(orc.get_state(), n, orc.S, orc.P)
    rng = np.random.default_rng(3)
    for e in range(n):
        rr, cc = np.nonzero(d["mat"][e] == 4)  # Foilage -> Scrub (depleted, regrows at p = 0.025)
        pick = rng.random(rr.size) < 0.9
        d["mat"][e, rr[pick], cc[pick]] = 3
    orc.set_state(join_state(d))
    eng = _engine(cfg, n, seed=0)
    eng.set_tasks(tl, None, assign)
    eng.set_state(orc.get_state())
    flips = 0
    for t in range(steps):
        acts = orc.scripted_actions(40 + t)
        orc.step(acts)
        eng.step(torch.from_numpy(acts).cuda())
        torch.cuda.synchronize()
        _cmp_state(eng.get_state(), orc.get_state(), n, eng.S, f"CanSeeTile step {t}")
        assert np.array_equal(eng.rew.cpu().numpy(), orc.rew), f"rewards @ {t}"
        flips += int((orc.rew[assign == 0] != 0).sum())  # Foilage came into / went out of view
    assert flips > 20, flips


def pathing_scenario(n=4):
    """SPEC §6 v2 window BFS under stress: in every env, hostile NPCs are put 2-7 tiles from live
    players and stone walls are scattered around them, so most hunts path around obstacles (and
    some targets are unreachable inside the window: greedy fallback). HIP vs oracle, bit-exact."""
    from oracle.oracle import join_state

    cfg = Config.preset("C3", MAP_N=4, early_stop_agent_num=0)
    orc = OracleEnvs(cfg, n, seed=41)
    orc.reset()
    for t in range(3):
        orc.step(orc.scripted_actions(t))
    d = split_state(orc.get_state(), n, orc.S, orc.P)
    rng = np.random.default_rng(12)
    F = abi.F
    for e in range(n):
        ent, mat = d["ent"][e], d["mat"][e]
        occupied = {(int(ent[F["row"], s]), int(ent[F["col"], s])) for s in range(orc.S) if ent[F["alive"], s]}
        players = [s for s in range(orc.P) if ent[F["alive"], s]]
        npcs = [s for s in range(orc.P, orc.S) if ent[F["alive"], s]][:60]
        for k, s in enumerate(npcs):
            p = players[k % len(players)]
            pr, pc = int(ent[F["row"], p]), int(ent[F["col"], p])
            for _ in range(50):
                r = int(np.clip(pr + rng.integers(-7, 8), 17, 142))
                c = int(np.clip(pc + rng.integers(-7, 8), 17, 142))
                if max(abs(r - pr), abs(c - pc)) >= 2 and (r, c) not in occupied and mat[r, c] not in (0, 1, 5, 14, 15):
                    break
            occupied.discard((int(ent[F["row"], s]), int(ent[F["col"], s])))
            occupied.add((r, c))
            ent[F["row"], s], ent[F["col"], s] = r, c
            ent[F["npc_type"], s] = 3
            ent[F["target_id"], s] = 0
        for p in players:  # scattered walls around each player, never under an entity
            pr, pc = int(ent[F["row"], p]), int(ent[F["col"], p])
            for _ in range(20):
                r, c = pr + int(rng.integers(-6, 7)), pc + int(rng.integers(-6, 7))
                if 16 <= r <= 143 and 16 <= c <= 143 and (r, c) not in occupied:
                    mat[r, c] = 5  # Stone
    orc.set_state(join_state(d))
    return orc


def test_npc_pathing_parity():
    """SPEC §6 v2 window BFS under stress (pathing_scenario): HIP vs oracle, bit-exact."""
    import torch

    n, steps = 4, 40
    F = abi.F
    orc = pathing_scenario(n)
    cfg = orc.config
    eng = _engine(cfg, n, seed=0)
    eng.set_state(orc.get_state())
    for t in range(steps):
        acts = orc.scripted_actions(300 + t)
        orc.step(acts)
        eng.step(torch.from_numpy(acts).cuda())
        torch.cuda.synchronize()
        _cmp_state(eng.get_state(), orc.get_state(), n, eng.S, f"pathing step {t}")
        assert np.array_equal(eng.rew.cpu().numpy(), orc.rew), f"rewards @ {t}"
        if t == 0:
            hunting = int((split_state(orc.get_state(), n, orc.S, orc.P)["ent"][:, F["target_id"]] > 0).sum())
            assert hunting > 100, hunting
    _cmp_events(eng, orc, n, "pathing end")


def test_curriculum_sampling_parity():
    """The reference's training curriculum (manual_curriculum.py + curriculum_tutorial.py, with
    PracticeEating), sampled per player by sampling_weight at every reset and auto-reset
    (nmmo_set_task_weights, SPEC §12): assignments, task state, rewards and Task obs bit-exact."""
    import torch

    from nmmo_amd import tasks

    n, steps = 6, 150
    cfg = Config.preset("C4", MAP_N=8, early_stop_agent_num=8)
    specs = tasks.manual_curriculum() + tasks.tutorial_curriculum()
    rng = np.random.default_rng(4)
    for s in specs:
        s.embedding = rng.standard_normal(cfg.TASK_EMBED_DIM).astype(np.float16)
    eng = _engine(cfg, n, seed=13)
    orc = OracleEnvs(cfg, n, seed=13)
    eng.set_curriculum(specs)
    orc.set_curriculum(specs)
    eng.reset()
    orc.reset()
    seen = set()
    for t in range(steps):
        acts = orc.scripted_actions(700 + t)
        orc.step(acts)
        eng.step(torch.from_numpy(acts).cuda())
        torch.cuda.synchronize()
        g = split_state(eng.get_state(), n, eng.S, eng.P)
        o = split_state(orc.get_state(), n, orc.S, orc.P)
        assert np.array_equal(g["tasks"], o["tasks"]), f"sampled assignment @ {t}"
        seen.update(np.unique(o["tasks"]).tolist())
        _cmp_state(eng.get_state(), orc.get_state(), n, eng.S, f"curriculum step {t}")
        assert np.array_equal(eng.rew.cpu().numpy(), orc.rew), f"rewards @ {t}"
        if t % 25 == 0:
            assert np.array_equal(eng.obs.cpu().numpy(), orc.obs), f"obs @ {t}"
    assert len(seen) > 200  # many distinct tasks drawn over the resets
    assert int(split_state(orc.get_state(), n, orc.S, orc.P)["env"][:, abi.E["episode"]].min()) >= 1


@pytest.mark.parametrize("P,N,preset", [(100, 50, "C4"), (13, 0, "C3"), (64, 256, "C4"), (1, 7, "C4")])
def test_rollout_parity_odd_sizes(P, N, preset):
    """Player/NPC counts that are not multiples of 8/16/64: scalar state-copy fallbacks, partial
    waves, partial 16-agent obs groups, tiny envs."""
    import torch

    n, steps = 3, 60
    cfg = Config.preset(preset, MAP_N=4, early_stop_agent_num=0, PLAYER_N=P, NPC_N=N)
    eng = _engine(cfg, n, seed=31)
    orc = OracleEnvs(cfg, n, seed=31)
    eng.reset()
    orc.reset()
    for t in range(steps):
        acts = orc.scripted_actions(300 + t)
        g_acts = eng.scripted_actions(300 + t)
        assert np.array_equal(g_acts.cpu().numpy(), acts), f"policy differs at step {t}"
        orc.step(acts)
        eng.step(torch.from_numpy(acts).cuda())
        torch.cuda.synchronize()
        _cmp_state(eng.get_state(), orc.get_state(), n, eng.S, f"P={P} N={N} step {t}", P=P)
        for name in ("rew", "term", "trunc", "mask"):
            assert np.array_equal(getattr(eng, name).cpu().numpy(), getattr(orc, name)), f"{name} @ {t}"
        _cmp_events(eng, orc, n, f"P={P} step {t}")
        if orc.obs is not None and t % 10 == 0:
            assert np.array_equal(eng.obs.cpu().numpy(), orc.obs), f"obs @ {t}"
