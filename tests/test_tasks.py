"""Task programs and rewards (SPEC.md §12): known answers on the CPU oracle, hand-computed from
the SPEC formulas. CPU only."""

import numpy as np
import pytest

from nmmo_amd import abi, tasks
from nmmo_amd.config import Config
from oracle.oracle import OracleEnvs, join_state, split_state
from tests.test_oracle import GRASS, SCRUB, WATER, find_tile, nbrs, noop_actions, park_others, place, put

F, E = abi.F, abi.E


def make(systems=("Resource",), P=4):
    cfg = Config(systems=systems, PLAYER_N=P, MAP_N=1, early_stop_agent_num=0)
    o = OracleEnvs(cfg, 1, seed=3)
    o.reset()
    return o, split_state(o.get_state(), 1, o.S, o.P)


def tstate(o):
    return split_state(o.get_state(), 1, o.S, o.P)["tstate"][0]


def test_count_event_progress_reward_and_completion():
    o, d = make()
    mat = d["mat"][0]
    r, c = find_tile(mat, lambda m, r, c: m[r, c] in (GRASS, SCRUB) and WATER in nbrs(m, r, c))
    park_others(d, {0}, mat)
    place(d, 0, r, c)
    put(o, d)
    o.set_tasks([tasks.task("CountEvent", event="DRINK_WATER", N=4)])
    rewards = []
    for _ in range(6):
        o.step(noop_actions(o))
        rewards.append(float(o.rew[0, 0]))
    assert rewards == [0.25, 0.25, 0.25, 0.25, 0.0, 0.0]  # one DRINK_WATER per tick, N = 4
    ts = tstate(o)[0]
    assert ts["last"] == 1.0 and ts["max_progress"] == 1.0 and ts["signals"] == 4
    assert ts["completed_tick"] == 4 and ts["acc"][0] == 6


def test_hoard_gold_can_go_down():
    o, d = make(systems=("Resource", "Item", "Exchange"))
    mat = d["mat"][0]
    r, c = find_tile(mat, lambda m, r, c: m[r, c] in (GRASS, SCRUB) and WATER not in nbrs(m, r, c))
    park_others(d, {0, 1}, mat)
    place(d, 0, r, c, gold=5)
    place(d, 1, r, c, gold=0)
    put(o, d)
    o.set_tasks([tasks.task("HoardGold", amount=10)])
    o.step(noop_actions(o))
    assert o.rew[0, 0] == np.float32(0.5)
    a = noop_actions(o)
    a[0, 0, 6] = 2  # GiveGold price index 2 -> amount 3, to player 1 (its visible row below)
    ent = split_state(o.get_state(), 1, o.S, o.P)["ent"][0]
    rows = sorted((ent[F["ds_row"], s], s) for s in range(o.S) if ent[F["alive"], s]
                  and max(abs(ent[F["row"], s] - r), abs(ent[F["col"], s] - c)) <= 7)
    a[0, 0, 7] = [s for _, s in rows].index(1)
    o.step(a)
    assert o.rew[0, 0] == np.float32(0.2 - 0.5)  # gold 5 -> 2: progress 0.5 -> 0.2
    assert o.rew[0, 1] == np.float32(0.3)         # player 1 also hoards: 0 -> 3


def test_weighted_sum_without_fma():
    o, d = make(systems=("Resource", "Item", "Equipment", "Profession"))
    mat = d["mat"][0]
    r, c = find_tile(mat, lambda m, r, c: m[r, c] in (GRASS, SCRUB) and WATER not in nbrs(m, r, c))
    park_others(d, {0}, mat)
    place(d, 0, r, c, fishing_exp=13)
    d["items"][0, 0, 0] = [8 | (1 << 5) | (1 << 9), 1 | (1 << 16)]  # Rod L1, equipped, row 1
    d["iring"][0, :] = np.r_[np.arange(2, 12 * o.P + 1), 0]
    d["env"][0, E["item_free_count"]] = 12 * o.P - 1
    put(o, d)
    o.set_tasks([tasks.practice_skill_with_tool("Fishing", 30)])
    o.step(noop_actions(o))
    want = np.float64(np.float32(0.3)) * 1.0 + np.float64(np.float32(0.7)) * (13 / 30)
    assert o.rew[0, 0] == np.float32(want)


def test_product_and_per_player_assignment_and_task_obs():
    cfg = Config.preset("C2", MAP_N=1, early_stop_agent_num=0, PLAYER_N=8)
    cfg.obs_layout = abi.OBS_FLAT
    o = OracleEnvs(cfg, 1, seed=5)
    emb = np.stack([np.full(cfg.TASK_EMBED_DIM, 0.5, np.float16), np.full(cfg.TASK_EMBED_DIM, -1, np.float16)])
    assign = np.array([[0, 1] * 4], np.int32)
    o.set_tasks([tasks.task("TickGE", num_tick=8), tasks.practice_inventory_management(12, 4)], emb, assign)
    o.reset()
    from nmmo_amd import layout

    t = layout.unflatten(o.obs)["Task"][0]
    assert np.all(t[0::2] == 0.5) and np.all(t[1::2] == -1.0)
    o.step(o.scripted_actions(0))
    alive = o.mask[0] == 1
    for p in range(8):
        if alive[p] and not o.term[0, p]:
            assert o.rew[0, p] == np.float32(1 / 8 if p % 2 == 0 else 1 / 4)


def test_builder_rejects_team_tasks_and_unknown_predicates():
    with pytest.raises(ValueError):
        tasks.task("AttainSkill", skill="Melee", level=3, num_agent=2)
    with pytest.raises(ValueError):
        tasks.task("CanSeeAgent", target="left_team")  # a team is a group, not an agent
    with pytest.raises(ValueError):
        tasks.task("CanSeeGroup", target="right_team_leader")
    with pytest.raises(ValueError):
        tasks.TaskSpec("TickGE", {"num_tick": 3}, reward_to="team")
    g = tasks.task("CanSeeGroup", target="left_team").term[0]
    assert (g.pred, g.a) == (abi.PRED["CanSeeGroup"], -1)
    assert tasks.task("CanSeeAgent", target=7).term[0].a == 7
    t = tasks.task("HarvestItem", item="Whetstone", level=2, quantity=3)
    assert (t.term[0].pred, t.term[0].a, t.term[0].b, t.term[0].c) == (abi.PRED["HarvestItem"], 13, 2, 3)


def _practice_eating_ref(n: int) -> float:
    """curriculum_tutorial.py:45-57 evaluated with Python floats, then norm() (clip to [0, 1])."""
    progress = n * 0.06
    if n >= 1:
        progress += 0.1
    if n >= 3:
        progress += 0.3
    return max(min(progress, 1.0), 0.0)


def test_practice_eating_progress_per_eat():
    """Known answer: an agent on Foilage eats once per tick; its progress after k eatings is the
    reference function's value, bit for bit (double), reward = the float32 of each increment."""
    o, d = make()
    mat = d["mat"][0]
    from tests.test_oracle import FOILAGE

    r, c = find_tile(mat, lambda m, r, c: m[r, c] == FOILAGE and WATER not in nbrs(m, r, c))
    park_others(d, {0}, mat)
    place(d, 0, r, c, food=5)
    put(o, d)
    o.set_tasks([tasks.practice_eating()])
    prev = 0.0
    for _ in range(3):
        o.step(noop_actions(o))
        ts = tstate(o)[0]
        n = int(ts["acc"][0])
        assert ts["last"] == _practice_eating_ref(n)
        assert o.rew[0, 0] == np.float32(ts["last"] - prev)
        prev = ts["last"]
    assert n >= 1


def test_practice_eating_reference_values():
    vals = [_practice_eating_ref(n) for n in range(13)]
    assert vals[0] == 0.0 and vals[1] == 0.06 + 0.1 and vals[10] == 1.0 and vals[12] == 1.0


def test_heldout_curriculum_matches_reference_names():
    """The 63 TaskSpecs of neurips23_evaluation/heldout_evaluation_task.py:30-138 built through
    nmmo_amd.tasks carry exactly the names stored in the reference's heldout .pkl, in order."""
    d = np.load("tests/golden/task_embeddings.npz")
    specs = tasks.heldout_curriculum()
    assert len(specs) == 63 == len(d["heldout_names"])
    assert [s.name for s in specs] == [str(x) for x in d["heldout_names"]]
    progs = [s.program() for s in specs]
    assert progs[0].term[0].pred == abi.PRED["TickGE"] and progs[0].term[0].a == 1024
    assert progs[2].term[0].pred == abi.PRED["DefeatEntity"] and progs[2].term[0].c == 20


def _visible(d, p, t):
    """t is in p's Entity obs: in the realm and among the first 100 visible by datastore row."""
    from tests.test_oracle import visible_index

    if not d["ent"][0, F["alive"], t]:
        return False
    try:
        return visible_index(d, p, t) < 100
    except ValueError:
        return False


def test_can_see_neighbouring_team_known_answer():
    """CanSeeAgent / CanSeeGroup (manual_curriculum.py:157-162) with SPEC §12's singleton teams
    in id order: agent i's left team is agent i - 1 (agent 1's is agent P), its right team agent
    i + 1 (agent P's is agent 1); progress 1 iff the target is in the agent's Entity obs after
    the tick. Players 0 and 3 stand 3 tiles apart, the others elsewhere."""
    from tests.test_oracle import plain

    o, d = make(P=4)
    mat = d["mat"][0]
    r, c = find_tile(mat, plain)
    r2, c2 = r + 3, c + 2
    park_others(d, {0, 3}, mat)
    place(d, 0, r, c)
    place(d, 3, r2, c2)
    put(o, d)
    tl = [tasks.task("CanSeeAgent", target="left_team_leader"), tasks.task("CanSeeGroup", target="right_team"),
          tasks.task("CanSeeAgent", target=1)]
    assign = np.array([[0, 1, 2, 1]], np.int32)
    o.set_tasks(tl, None, assign)
    o.step(noop_actions(o))
    d = split_state(o.get_state(), 1, o.S, o.P)
    P = 4
    target = {0: P - 1, 1: 2, 2: 0, 3: 0}  # slots: left of id 1 = id 4; right of id 2 = id 3; agent 1; right of id 4 = id 1
    for p in range(P):
        want = 1.0 if _visible(d, p, target[p]) else 0.0
        assert float(o.rew[0, p]) == want, (p, want)
    assert o.rew[0, 0] == 1.0 and o.rew[0, 3] == 1.0  # the pair that stands together


def test_sample_eval_curriculum_matches_reference_specs():
    """The 24 TaskSpecs of neurips23_evaluation/sample_evaluation_task.py:12-52 in the order and
    with the arguments the reference's sample_eval_task_with_embedding.pkl holds them (read off
    its opcode stream, tests/golden/make_task_fixtures.py), so its 24 embeddings attach in order."""
    import json

    d = np.load("tests/golden/task_embeddings.npz")
    ref = json.loads(str(d["sample_specs"]))
    specs = tasks.sample_eval_curriculum()
    assert [[s.eval_fn, s.eval_fn_kwargs, s.sampling_weight] for s in specs] == ref
    assert len(specs) == d["sample_emb"].shape[0] == 24
    for s, e in zip(specs, d["sample_emb"]):
        s.embedding = e
        s.program()
    held = json.loads(str(d["heldout_specs"]))
    assert [[s.eval_fn, s.eval_fn_kwargs, s.sampling_weight] for s in tasks.heldout_curriculum()] == held


def test_manual_and_tutorial_curricula_build():
    m = tasks.manual_curriculum()
    assert len(m) <= abi.MAX_TASKS
    assert all(s.sampling_weight > 0 for s in m)
    for s in m + tasks.tutorial_curriculum():
        s.program()
    names = [s.name for s in m]
    assert "Task_PracticeSkillWithTool_(skill:Fishing_exp:50)_reward_to:agent" in names
    for t in ["left_team_leader", "right_team_leader"]:
        assert f"Task_CanSeeAgent_(target:{t})_reward_to:agent" in names
    for t in ["left_team", "right_team"]:
        assert f"Task_CanSeeGroup_(target:{t})_reward_to:agent" in names
    i = names.index("Task_OccupyTile_(row:80_col:80)_reward_to:agent")
    assert names[i + 1].startswith("Task_CanSeeAgent") and names[i + 5].startswith("Task_ScoreHit")
    assert len(set(names)) == len(names)


def test_sampling_by_weight_on_every_reset():
    """nmmo_set_task_weights on the oracle: assignments drawn per player at reset and at each
    auto-reset, frequencies follow the weights, zero weight never drawn."""
    cfg = Config.preset("C2", MAP_N=2, early_stop_agent_num=8)
    o = OracleEnvs(cfg, 16, seed=9)
    specs = [tasks.TaskSpec("TickGE", {"num_tick": 1024}, sampling_weight=3.0),
             tasks.TaskSpec("CountEvent", {"event": "EAT_FOOD", "N": 5}, sampling_weight=1.0),
             tasks.TaskSpec("PracticeEating", {}, sampling_weight=0.0)]
    o.set_curriculum(specs)
    o.reset()
    a0 = split_state(o.get_state(), 16, o.S, o.P)["tasks"].copy()
    counts = np.bincount(a0.ravel(), minlength=3)
    assert counts[2] == 0
    assert abs(counts[0] / counts.sum() - 0.75) < 0.05
    o.end_episodes(np.ones(16, np.uint8))
    o.step(o.scripted_actions(0))  # auto-reset: a fresh draw (new episode seed)
    a1 = split_state(o.get_state(), 16, o.S, o.P)["tasks"]
    assert not np.array_equal(a0, a1)
    with pytest.raises(ValueError):
        o.set_task_weights([1.0, 2.0])  # wrong length
    with pytest.raises(ValueError):
        o.set_task_weights([0.0, 0.0, 0.0])
