"""Protocol 1 facade (nmmo.Env shape, nmmo_amd/vecenv.py) against every attribute path the
reference's BaseStatWrapper reads (reinforcement_learning/stat_wrapper.py:122-185) and
train_helper.py:133-225 reads, built from a CPU-oracle state blob (the same nmmo_get_state
layout the GPU engine returns). CPU only; the GPU NmmoEnv runs the same walk in
tests/test_gpu_vecenv.py."""

import numpy as np

from nmmo_amd import abi, tasks
from nmmo_amd.config import Config
from nmmo_amd.vecenv import EventLog, Val, _Realm, parse_env_state, tasks_from_state
from oracle.oracle import OracleEnvs


def walk_stat_wrapper_reads(realm, agent_task_map, agent_id, terminated):
    """The reads of stat_wrapper.py:122-185 for one finished agent, in order; returns the stats."""
    info = {"stats": {}}
    tick_log = realm.event_log.get_data(agents=[agent_id], tick=-1)  # :123
    assert tick_log.ndim == 2 and tick_log.shape[1] == abi.EVENT_COLS
    agent = realm.players.dead_this_tick.get(agent_id, realm.players.get(agent_id))  # :136
    assert agent is not None  # :137
    info["length"] = realm.tick  # :140
    if terminated:  # :145-148
        info["stats"]["cod/attacked"] = 1.0 if agent.damage.val > 0 else 0.0
        info["stats"]["cod/starved"] = 1.0 if agent.food.val == 0 else 0.0
        info["stats"]["cod/dehydrated"] = 1.0 if agent.water.val == 0 else 0.0
    task = agent_task_map[agent_id][0]  # :155
    info["stats"]["task/completed"] = 1.0 if task.completed else 0.0
    info["stats"]["task/pcnt_2_reward_signal"] = 1.0 if task.reward_signal_count >= 2 else 0.0
    info["stats"]["task/pcnt_0p2_max_progress"] = 1.0 if task._max_progress >= 0.2 else 0.0
    info["curriculum"] = {task.spec_name: (task._max_progress, task.reward_signal_count)}
    info["stats"]["achieved/max_combat_level"] = agent.attack_level  # :170
    info["stats"]["achieved/max_harvest_skill_ammo"] = max(
        agent.prospecting_level.val, agent.carving_level.val, agent.alchemy_level.val)
    info["stats"]["achieved/max_harvest_skill_consum"] = max(
        agent.fishing_level.val, agent.herbalism_level.val)
    log = realm.event_log.get_data(agents=[agent_id])  # process_event_log :218-219
    col = realm.event_log.attr_to_col
    for k in ("event", "item_type", "level", "distance", "gold", "damage", "target_ent"):
        log[:, col[k]]
    return info


def test_facade_walk_over_oracle_state():
    cfg = Config.preset("C4", MAP_N=2, early_stop_agent_num=0)
    o = OracleEnvs(cfg, 1, seed=17)
    specs = tasks.heldout_curriculum()
    o.set_curriculum(specs)
    o.reset()
    names = [s.name for s in specs]
    possible = list(range(1, cfg.PLAYER_N + 1))
    walked_dead = walked_alive = 0
    for t in range(120):
        o.step(o.scripted_actions(40 + t))
        st = parse_env_state(o.get_state(), o.S, o.P)
        realm = _Realm(st, o.events(0))
        if realm.tick == 0:  # the auto-reset step of a finished episode
            continue
        tmap = {tk.assignee[0]: [tk] for tk in tasks_from_state(st, possible, names)}
        died = [a for a in possible if o.term[0, a - 1]]
        # every agent culled this tick is in dead_this_tick, none of them among the live players
        assert sorted(realm.players.dead_this_tick) == sorted(died)
        assert not set(died) & set(realm.players)
        for a in died:
            info = walk_stat_wrapper_reads(realm, tmap, a, terminated=True)
            ag = realm.players.dead_this_tick[a]
            assert info["stats"]["cod/starved"] == (1.0 if int(ag.food) == 0 else 0.0)
            assert info["length"] == realm.tick
            walked_dead += 1
        for a in list(realm.players)[:2]:
            walk_stat_wrapper_reads(realm, tmap, a, terminated=False)
            walked_alive += 1
    assert walked_dead > 0 and walked_alive > 0


def test_val_attributes_and_task_fields():
    v = Val(7)
    assert v == 7 and v.val == 7 and v + 1 == 8 and isinstance(v.val, int)
    cfg = Config.preset("C3", MAP_N=1)
    o = OracleEnvs(cfg, 1, seed=2)
    o.reset()
    st = parse_env_state(o.get_state(), o.S, o.P)
    realm = _Realm(st, np.zeros((0, abi.EVENT_COLS), np.int32))
    p1 = realm.players[1]
    assert p1.attack_level == max(p1.melee_level, p1.range_level, p1.mage_level) == 1
    assert p1.health.val == 100 and p1.name == "Player_1"
    assert all(n < 0 for n in realm.npcs)
    ts = tasks_from_state(st, list(range(1, o.P + 1)), [tasks.spec_name("TickGE", num_tick=1024)])
    assert ts[0].spec_name == "Task_TickGE_(num_tick:1024)_reward_to:agent"
    assert ts[0].completed is False and ts[0].reward_signal_count == 0 and ts[0]._max_progress == 0.0
    assert set(ts[0].progress_info) == {"max_progress", "completed_tick"}
    assert isinstance(realm.event_log, EventLog)


def test_agent_from_env_creator_closure():
    """GpuVecEnv picks the device RewardWrapper from the class environment.make_env_creator
    closed over (environment.py:50-58, train.py:226), so the default train.py needs no extra
    argument; a Syllabus creator is refused (curricula go through set_curriculum)."""
    import pytest

    from nmmo_amd.vecenv import _as_dict, agent_from_creator

    def make_env_creator(reward_wrapper_cls, syllabus_wrapper=False, syllabus=None):  # environment.py:50
        def env_creator(*args, **kwargs):
            return reward_wrapper_cls, syllabus_wrapper, syllabus
        return env_creator

    RW = type("RewardWrapper", (), {"__module__": "agent_zoo.takeru.reward_wrapper"})
    assert agent_from_creator(make_env_creator(RW)) == "takeru"
    assert agent_from_creator(make_env_creator(type("X", (), {}))) is None
    assert agent_from_creator(None) is None
    with pytest.raises(ValueError, match="Syllabus"):
        agent_from_creator(make_env_creator(RW, syllabus=object()))
    from types import SimpleNamespace

    assert _as_dict(SimpleNamespace(eval_mode=False, early_stop_agent_num=8)) == {
        "eval_mode": False, "early_stop_agent_num": 8}


def test_obs_writes_follow_the_agent_policy():
    """GpuVecEnv's obs contract defaults to what the named agent's policy writes into its input in
    place: the start-kit TileEncoder's Tile edit (baseline_policy.py:96-97) scopes the rewrite to the
    Tile sections; takeru / yaofeng write nothing; without an agent every row is rewritten."""
    from nmmo_amd.vecenv import resolve_obs_writes

    assert resolve_obs_writes("neurips23_start_kit") == frozenset({"Tile"})
    assert resolve_obs_writes("takeru") == resolve_obs_writes("yaofeng") == frozenset()
    assert resolve_obs_writes(None) == "all"
    assert resolve_obs_writes(None, obs_readonly=True) == frozenset()
    assert resolve_obs_writes("takeru", obs_writes="all") == "all"
    assert resolve_obs_writes(None, obs_writes={"Tile", "Entity"}) == frozenset({"Tile", "Entity"})
    import pytest

    with pytest.raises(ValueError):
        resolve_obs_writes(None, obs_writes={"Tiles"})
    with pytest.raises(ValueError):
        resolve_obs_writes(None, obs_writes="Tile")
