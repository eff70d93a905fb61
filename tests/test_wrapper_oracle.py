"""The CPU restatement of the reference's wrappers (oracle/wrapper.py, SPEC.md §13) on hand
cases from stat_wrapper.py's rules, and the host-side info/config helpers of nmmo_amd.wrappers.
CPU only."""

import numpy as np
import pytest

from nmmo_amd import abi
from nmmo_amd.config import Config
from nmmo_amd.wrappers import AGENTS, info_dict, wrapper_config
from oracle.oracle import OracleEnvs
from oracle.wrapper import OracleWrapper, count_unique_events, process_event_log

EC = abi.EventCode


def row(ent, tick, code, type_=0, level=0, number=0, gold=0, target=0, i=0):
    return [i, ent, tick, code, type_, level, number, gold, target]


def test_count_unique_events_rules():
    # stat_wrapper.py:296-310: new tuples count once; PLAYER_KILL / EARN_GOLD always count
    log = np.array([row(1, 1, EC.EAT_FOOD), row(1, 1, EC.EAT_FOOD), row(1, 1, EC.PLAYER_KILL, 0, 3),
                    row(1, 1, EC.PLAYER_KILL, 0, 3), row(1, 1, EC.EARN_GOLD, 5, 1, 1, 9),
                    row(1, 1, EC.EARN_GOLD, 5, 1, 1, 4), row(1, 1, EC.HARVEST_ITEM, 16, 1)], np.int32)
    seen = set()
    assert count_unique_events(log, seen) == 1 + 2 + 2 + 1
    assert count_unique_events(log[:2], seen) == 0  # EAT_FOOD already experienced
    assert count_unique_events(np.zeros((0, 9), np.int32), seen) == 0


def test_process_event_log_hand_case():
    log = np.array([
        row(3, 1, EC.GO_FARTHEST, number=5), row(3, 2, EC.GO_FARTHEST, number=9),
        row(3, 2, EC.SCORE_HIT, 1, 0, 7), row(3, 3, EC.SCORE_HIT, 2, 0, 12),
        row(3, 3, EC.EARN_GOLD, gold=4), row(3, 4, EC.EARN_GOLD, gold=6),
        row(3, 4, EC.HARVEST_ITEM, 14, 2), row(3, 4, EC.LOOT_ITEM, 3, 5), row(3, 5, EC.BUY_ITEM, 14, 4),
        row(3, 5, EC.EQUIP_ITEM, 9, 1), row(3, 6, EC.PLAYER_KILL, 0, 2, target=-4),
        row(3, 6, EC.PLAYER_KILL, 0, 1, target=7), row(3, 6, EC.HARVEST_ITEM, 5, 1)], np.int32)
    ach, perf = process_event_log(log)
    assert ach["achieved/max_progress_to_center"] == 9
    assert ach["achieved/earned_gold"] == 10
    assert ach["achieved/max_damage"] == 12
    assert ach["achieved/max_ammo_level"] == 4 and ach["achieved/max_armor_level"] == 5
    assert ach["achieved/max_weapon_level"] == 1 and "achieved/max_tool_level" not in ach
    assert ach["achieved/agent_kill_count"] == 1 and ach["achieved/npc_kill_count"] == 1
    assert perf["event/equip_tool"] and not perf["event/equip_armor"] and perf["event/harvest_weapon"]
    assert perf["event/score_hit"] and not perf["event/eat_food"]


def test_wrapper_config_follows_reference_signatures():
    c = wrapper_config("neurips23_start_kit", heal_bonus_weight=0.03, explore_bonus_weight=0.01,
                       eval_mode=False, early_stop_agent_num=8, use_custom_reward=True)
    assert (c.kind, c.heal_bonus_weight, c.explore_bonus_weight, c.clip_unique_event) == \
        (abi.WRAP_START_KIT, 0.03, 0.01, 3)
    y = wrapper_config("yaofeng")
    assert y.disable_give == 1 and y.donot_attack_dangerous_npc == 1 and y.custom_bonus_scale == 1.0
    assert wrapper_config("takeru").disable_give == 1
    assert wrapper_config("base", use_custom_reward=False).use_custom_reward == 0
    with pytest.raises(TypeError):
        wrapper_config("takeru", heal_bonus_weight=1.0)
    with pytest.raises(ValueError):
        wrapper_config("yaofeng", randomize_spawn_immunity=True)
    assert set(AGENTS) >= {"neurips23_start_kit", "takeru", "yaofeng", "hybrid"}


def test_info_dict_keys_match_base_stat_wrapper():
    rec = np.zeros((), abi.agent_info_dtype())
    rec["done"], rec["length"], rec["ret"], rec["max_progress"] = 1, 40, 0.25, 0.5
    rec["reward_signal_count"], rec["cod_starved"], rec["performed"] = 3, 1, 0b1000000000011
    rec["max_item_level"] = [-1, 2, -1, -1, 1]
    info = info_dict(rec, "TickGE_1024")
    s = info["stats"]
    assert info["length"] == 40 and info["return"] == 0.25
    assert info["curriculum"] == {"TickGE_1024": (0.5, 3)}
    assert s["cod/starved"] == 1.0 and s["task/pcnt_2_reward_signal"] == 1.0
    assert s["task/pcnt_0p2_max_progress"] == 1.0 and s["task/completed"] == 0.0
    assert s["event/eat_food"] == 1.0 and s["event/drink_water"] == 1.0 and s["event/harvest_weapon"] == 1.0
    assert s["achieved/max_weapon_level"] == 2.0 and "achieved/max_armor_level" not in s
    assert info_dict(rec, stat_prefix="learner").keys() == {"learner"}


@pytest.mark.parametrize("agent,kw", [
    ("neurips23_start_kit", dict(heal_bonus_weight=0.03, explore_bonus_weight=0.01)),
    ("yaofeng", dict(hp_bonus_weight=0.01, gold_bonus_weight=0.1)),
])
def test_oracle_wrapper_rollout(agent, kw):
    cfg = Config.preset("C4", MAP_N=4, early_stop_agent_num=8, HORIZON=60)
    envs = OracleEnvs(cfg, 2, seed=9)
    raw = OracleEnvs(cfg, 2, seed=9)
    ow = OracleWrapper(envs, agent, **kw)
    envs.reset()
    raw.reset()
    ow.after_reset()
    done, shaped = 0, 0
    for t in range(70):
        a = raw.scripted_actions(t)
        envs.step(a)
        raw.step(a)
        ow.after_step(a)
        shaped += int(np.sum(envs.rew != raw.rew))
        for e in range(2):
            for ag, info in ow.infos[e].items():
                done += 1
                assert info["length"] >= 1 and "achieved/unique_events" in info["stats"]
                assert raw.term[e, ag - 1] or raw.trunc[e, ag - 1]
        if envs.obs is not None and agent == "neurips23_start_kit":
            lay = ow.lay["ActionTargets.Sell.Price"]
            for e in range(2):
                for p in range(cfg.PLAYER_N):
                    if envs.mask[e, p] and envs.obs[e, p].any():
                        assert envs.obs[e, p, lay.offset + ow.hist[e][p + 1]["prev_price"]] == 0
    assert done > 0 and shaped > 0
