"""The reference's env wrappers on the device (SPEC.md §13, nmmo_set_wrapper).

`env_creator` wraps every nmmo.Env in the agent's RewardWrapper(BaseStatWrapper)
(reinforcement_learning/environment.py:58) with the YAML `reward_wrapper:` kwargs
(config.yaml:99-107 + the agent section). `wrapper_config(agent, **kwargs)` takes the same
kwargs and returns the C struct; `info_dict(rec)` turns an episode record (NmmoAgentInfo) back
into the info dict BaseStatWrapper builds (stat_wrapper.py:128-185), key for key.
"""

from __future__ import annotations

import numpy as np

from . import abi

# constructor defaults of each RewardWrapper (agent_zoo/<agent>/reward_wrapper.py __init__)
AGENTS = {
    "base": dict(kind=abi.WRAP_BASE),
    "neurips23_start_kit": dict(kind=abi.WRAP_START_KIT, heal_bonus_weight=0.0,
                                explore_bonus_weight=0.0, clip_unique_event=3),
    "takeru": dict(kind=abi.WRAP_TAKERU, explore_bonus_weight=0.0, clip_unique_event=3,
                   disable_give=True),
    "yaofeng": dict(kind=abi.WRAP_YAOFENG, hp_bonus_weight=0.0, exp_bonus_weight=0.0,
                    defense_bonus_weight=0.0, attack_bonus_weight=0.0, gold_bonus_weight=0.0,
                    custom_bonus_scale=1.0, randomize_spawn_immunity=False, disable_give=True,
                    donot_attack_dangerous_npc=True),
}
AGENTS["hybrid"] = AGENTS["yaofeng"]  # agent_zoo/hybrid.py re-exports yaofeng's RewardWrapper
# BaseStatWrapper arguments (stat_wrapper.py:10-17); early_stop_agent_num lives in Config
_BASE_KEYS = {"eval_mode", "early_stop_agent_num", "stat_prefix", "use_custom_reward"}


def wrapper_config(agent: str = "neurips23_start_kit", **kwargs) -> abi.NmmoWrapperConfig:
    """The C wrapper config for `agent`'s RewardWrapper built with `kwargs` (the reference's
    `reward_wrapper` section, e.g. heal_bonus_weight=0.03, explore_bonus_weight=0.01)."""
    if agent not in AGENTS:
        raise ValueError(f"unknown agent {agent!r} (one of {sorted(AGENTS)})")
    d = dict(AGENTS[agent])
    kind = d.pop("kind")
    for k, v in kwargs.items():
        if k in _BASE_KEYS:
            continue
        if k not in d:
            raise TypeError(f"{agent} RewardWrapper has no argument {k!r}")
        d[k] = v
    if d.pop("randomize_spawn_immunity", False):
        raise ValueError("randomize_spawn_immunity is not implemented by the reference either (TODO there)")
    c = abi.NmmoWrapperConfig()
    c.kind = kind
    c.use_custom_reward = int(bool(kwargs.get("use_custom_reward", True)))
    c.eval_mode = int(bool(kwargs.get("eval_mode", False)))
    c.clip_unique_event = int(d.pop("clip_unique_event", 3))
    c.disable_give = int(bool(d.pop("disable_give", False)))
    c.donot_attack_dangerous_npc = int(bool(d.pop("donot_attack_dangerous_npc", False)))
    c.custom_bonus_scale = float(d.pop("custom_bonus_scale", 1.0))
    for k, v in d.items():
        setattr(c, k, float(v))
    return c


def info_dict(rec, task_name: str = "task", stat_prefix: str | None = None) -> dict:
    """BaseStatWrapper's info for an agent's final step from its NmmoAgentInfo record
    (a row of abi.agent_info_dtype())."""
    stats = {
        "cod/attacked": float(rec["cod_attacked"]),
        "cod/starved": float(rec["cod_starved"]),
        "cod/dehydrated": float(rec["cod_dehydrated"]),
        "task/completed": 1.0 if rec["task_completed"] else 0.0,
        "task/pcnt_2_reward_signal": 1.0 if rec["reward_signal_count"] >= 2 else 0.0,
        "task/pcnt_0p2_max_progress": 1.0 if rec["max_progress"] >= 0.2 else 0.0,
        "achieved/max_combat_level": int(rec["max_combat_level"]),
        "achieved/max_harvest_skill_ammo": int(rec["max_harvest_skill_ammo"]),
        "achieved/max_harvest_skill_consum": int(rec["max_harvest_skill_consum"]),
    }
    achieved = {
        "achieved/max_progress_to_center": int(rec["max_progress_to_center"]),
        "achieved/earned_gold": int(rec["earned_gold"]),
        "achieved/max_damage": int(rec["max_damage"]),
    }
    for k, cat in enumerate(abi.ITEM_CATEGORIES):
        if rec["max_item_level"][k] >= 0:
            achieved[f"achieved/max_{cat}_level"] = int(rec["max_item_level"][k])
    achieved["achieved/agent_kill_count"] = int(rec["agent_kill_count"])
    achieved["achieved/npc_kill_count"] = int(rec["npc_kill_count"])
    achieved["achieved/unique_events"] = int(rec["unique_events"])
    performed = {f"event/{name}": bool((int(rec["performed"]) >> b) & 1)
                 for b, name in enumerate(abi.PERFORMED_KEYS)}
    for k, v in list(achieved.items()) + list(performed.items()):
        stats[k] = float(v)
    info = {"stats": stats, "length": int(rec["length"]), "return": float(rec["ret"]),
            "curriculum": {task_name: (float(rec["max_progress"]), int(rec["reward_signal_count"]))}}
    return {stat_prefix: info} if stat_prefix else info


def infos_from_records(records: np.ndarray, task_names=None, stat_prefix=None) -> list:
    """records: agent_info_dtype [n_envs, P] -> per env {agent_id: info} for the agents whose
    episode ended this step (the per-env info dicts a pufferlib pool hands to the trainer)."""
    out = []
    for e in range(records.shape[0]):
        d = {}
        for a in np.nonzero(records["done"][e])[0]:
            name = task_names[e][a] if task_names is not None else "task"
            d[int(a) + 1] = info_dict(records[e, a], name, stat_prefix)
        out.append(d)
    return out
