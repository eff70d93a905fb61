"""TEST INFRASTRUCTURE ONLY — CPU restatement of the reference's env wrappers (SPEC.md §13).

Only tests/ may import this module. It follows the reference's own Python, which (unlike the
simulator) is in /root/reference, so these rules are pinned to readable code:
  BaseStatWrapper          reinforcement_learning/stat_wrapper.py:9-185
  process_event_log        reinforcement_learning/stat_wrapper.py:216-293
  count_unique_events      reinforcement_learning/stat_wrapper.py:296-310
  start-kit RewardWrapper  agent_zoo/neurips23_start_kit/reward_wrapper.py:25-82
  takeru RewardWrapper     agent_zoo/takeru/reward_wrapper.py:25-51
  yaofeng RewardWrapper    agent_zoo/yaofeng/reward_wrapper.py:49-127
It keeps the reference's data structures (per-agent dicts, a Python `set` of event tuples, the
agent's whole episode log scanned with numpy at its final step) on top of the oracle env's
state and event log — an algorithm independent of the GPU's per-tick bitset/accumulator pass.
"""

from __future__ import annotations

import numpy as np

from nmmo_amd import abi
from nmmo_amd.layout import flat_layout

from .oracle import split_state

EC = abi.EventCode
COL = abi.ATTR_TO_COL
# stat_wrapper.py:190-192 over nmmo's EventCode names
INFO_KEY_TO_EVENT_CODE = {"event/" + k.lower(): v for k, v in vars(EC).items() if k.isupper()}
KEY_EVENT = ["eat_food", "drink_water", "score_hit", "player_kill", "consume_item", "harvest_item",
             "list_item", "buy_item"]
# nmmo.systems.item ARMOR / WEAPON / TOOL / AMMUNITION / CONSUMABLE type ids (SPEC §9)
ITEM_TYPE = {"armor": [2, 3, 4], "weapon": [5, 6, 7], "tool": [8, 9, 10, 11, 12],
             "ammo": [13, 14, 15], "consumable": [16, 17]}
EVERY_EVENT_TO_COUNT = {EC.PLAYER_KILL, EC.EARN_GOLD}
SKILLS = ["melee", "range", "mage", "fishing", "herbalism", "prospecting", "carving", "alchemy"]
F = abi.F


def count_unique_events(tick_log, experienced):
    n = 0
    for row in tick_log[:, 3:6]:
        ev = tuple(int(x) for x in row)
        if ev not in experienced:
            experienced.add(ev)
            n += 1
        elif row[0] in EVERY_EVENT_TO_COUNT:
            n += 1
    return n


def process_event_log(log):
    """achieved, performed of an agent's episode log (stat_wrapper.py:216-293)."""
    ev = log[:, COL["event"]]
    cnt = {k: int(np.sum(ev == c)) for k, c in INFO_KEY_TO_EVENT_CODE.items()}
    performed = {"event/" + e: cnt["event/" + e] > 0 for e in KEY_EVENT}
    for t, ids in ITEM_TYPE.items():
        if t == "consumable":
            continue
        performed["event/equip_" + t] = np.sum((ev == EC.EQUIP_ITEM) & np.isin(log[:, COL["item_type"]], ids)) > 0
    performed["event/harvest_weapon"] = np.sum(
        (ev == EC.HARVEST_ITEM) & np.isin(log[:, COL["item_type"]], ITEM_TYPE["weapon"])) > 0
    achieved = {}
    idx = ev == EC.GO_FARTHEST
    achieved["achieved/max_progress_to_center"] = int(np.max(log[idx, COL["distance"]])) if idx.sum() else 0
    idx = ev == EC.EARN_GOLD
    achieved["achieved/earned_gold"] = int(np.sum(log[idx, COL["gold"]]))
    idx = ev == EC.SCORE_HIT
    achieved["achieved/max_damage"] = int(np.max(log[idx, COL["damage"]])) if idx.sum() else 0
    idx = np.isin(ev, [EC.HARVEST_ITEM, EC.LOOT_ITEM, EC.BUY_ITEM])
    if idx.sum():
        for t, ids in ITEM_TYPE.items():
            sel = np.isin(log[idx, COL["item_type"]], ids)
            if sel.sum():
                achieved["achieved/max_" + t + "_level"] = int(np.max(log[idx][sel, COL["level"]]))
    idx = ev == EC.PLAYER_KILL
    achieved["achieved/agent_kill_count"] = int(np.sum(idx & (log[:, COL["target_ent"]] > 0)))
    achieved["achieved/npc_kill_count"] = int(np.sum(idx & (log[:, COL["target_ent"]] < 0)))
    achieved["achieved/unique_events"] = count_unique_events(log, set())
    return achieved, performed


class OracleWrapper:
    """The wrapper pass over an OracleEnvs batch: call `after_step(actions)` after every
    `envs.step(actions)` and `after_reset()` after `envs.reset()`. Rewards (envs.rew) and obs
    (envs.obs) are edited in place; `self.infos[e]` = {agent_id: info} of the last step."""

    def __init__(self, envs, agent="neurips23_start_kit", **kw):
        from nmmo_amd.wrappers import AGENTS

        self.envs = envs
        self.agent = agent
        d = dict(AGENTS[agent])
        self.kind = d.pop("kind")
        self.eval_mode = bool(kw.pop("eval_mode", False))
        self.use_custom_reward = bool(kw.pop("use_custom_reward", True))
        kw.pop("early_stop_agent_num", None)
        kw.pop("stat_prefix", None)
        d.update(kw)
        self.w = d
        self.P = envs.P
        self.ids = list(range(1, self.P + 1))
        self.lay = flat_layout(envs.config.TASK_EMBED_DIM)
        self.infos = [{} for _ in range(envs.n_envs)]
        for e in range(envs.n_envs):
            self._reset_env(e)

    # -- BaseStatWrapper._reset_episode_stats + RewardWrapper._reset_reward_vars
    def _reset_env(self, e):
        if not hasattr(self, "cum"):
            n = self.envs.n_envs
            self.cum, self.uniq, self.hist, self.data, self.log = ([None] * n for _ in range(5))
        self.cum[e] = {a: 0 for a in self.ids}
        self.uniq[e] = {a: {"experienced": set(), "prev_count": 0, "curr_count": 0} for a in self.ids}
        self.hist[e] = {a: {"prev_price": 0, "prev_moves": []} for a in self.ids}
        self.data[e] = {a: {"hp": 100, "exp": 0, "damage_received": 0, "damage_inflicted": 0, "gold": 0}
                        for a in self.ids}
        self.log[e] = np.zeros((0, abi.EVENT_COLS), np.int32)

    def after_reset(self):
        st = self._state()
        for e in range(self.envs.n_envs):
            self._reset_env(e)
            self.infos[e] = {}
            self._observation(e, st, self.envs.mask[e])

    def _state(self):
        return split_state(self.envs.get_state(), self.envs.n_envs, self.envs.S, self.P)

    def after_step(self, actions):
        st = self._state()
        for e in range(self.envs.n_envs):
            tick = int(st["env"][e][abi.E["tick"]])
            self.infos[e] = {}
            if tick == 0:  # pufferlib auto-reset happened in this step
                self._reset_env(e)
                self._observation(e, st, self.envs.mask[e])
                continue
            rows = self.envs.events(e)
            rows = rows[rows[:, COL["tick"]] == tick]
            self.log[e] = np.concatenate([self.log[e], rows])
            present = [a for a in self.ids if self.envs.mask[e, a - 1]]
            # action(): before env.step in the reference, for the agents alive at step start
            for a in present:
                self.hist[e][a]["prev_price"] = int(actions[e, a - 1, 10])
                self.hist[e][a]["prev_moves"].append(int(actions[e, a - 1, 8]))
            for a in present:
                rew = float(self.envs.rew[e, a - 1])
                term = bool(self.envs.term[e, a - 1])
                trunc = bool(self.envs.trunc[e, a - 1])
                trunc, info = self._process_stats(e, st, a, tick, rows, rew, term, trunc)
                if self.use_custom_reward:
                    rew = self._shape(e, st, a, rew, term, trunc)
                else:
                    rew = 0 if term is True else rew
                self.envs.rew[e, a - 1] = np.float32(rew)
                if info:
                    self.infos[e][a] = info
            self._observation(e, st, self.envs.mask[e])

    def _ent(self, st, e, a, field):
        return int(st["ent"][e][F[field]][a - 1])

    def _process_stats(self, e, st, a, tick, rows, reward, terminated, truncated):
        info = {}
        tick_log = rows[rows[:, COL["ent_id"]] == a]
        u = self.uniq[e][a]
        u["prev_count"] = u["curr_count"]
        u["curr_count"] += count_unique_events(tick_log, u["experienced"])
        if not (terminated or truncated):
            self.cum[e][a] += reward
            return truncated, info
        info["stats"] = {}
        info["length"] = tick
        info["return"] = self.cum[e][a]
        if terminated:
            info["stats"]["cod/attacked"] = 1.0 if self._ent(st, e, a, "damage") > 0 else 0.0
            info["stats"]["cod/starved"] = 1.0 if self._ent(st, e, a, "food") == 0 else 0.0
            info["stats"]["cod/dehydrated"] = 1.0 if self._ent(st, e, a, "water") == 0 else 0.0
        else:
            info["stats"]["cod/attacked"] = 0
            info["stats"]["cod/starved"] = 0
            info["stats"]["cod/dehydrated"] = 0
        ts = st["tstate"][e][a - 1]
        completed = int(ts["completed_tick"]) != 0
        maxp, signals = float(ts["max_progress"]), int(ts["signals"])
        info["stats"]["task/completed"] = 1.0 if completed else 0.0
        info["stats"]["task/pcnt_2_reward_signal"] = 1.0 if signals >= 2 else 0.0
        info["stats"]["task/pcnt_0p2_max_progress"] = 1.0 if maxp >= 0.2 else 0.0
        info["curriculum"] = {"task": (maxp, signals)}
        if self.eval_mode:
            info["return"] = maxp
        lv = {s: self._ent(st, e, a, s + "_level") for s in SKILLS}
        info["stats"]["achieved/max_combat_level"] = max(lv["melee"], lv["range"], lv["mage"])
        info["stats"]["achieved/max_harvest_skill_ammo"] = max(lv["prospecting"], lv["carving"], lv["alchemy"])
        info["stats"]["achieved/max_harvest_skill_consum"] = max(lv["fishing"], lv["herbalism"])
        log = self.log[e][self.log[e][:, COL["ent_id"]] == a]
        achieved, performed = process_event_log(log)
        for k, v in list(achieved.items()) + list(performed.items()):
            info["stats"][k] = float(v)
        return truncated, info

    def _shape(self, e, st, a, reward, terminated, truncated):
        w = self.w
        done = terminated or truncated
        u = self.uniq[e][a]

        def explore():
            if w["explore_bonus_weight"] > 0 and u["curr_count"] > u["prev_count"]:
                return min(w["clip_unique_event"], u["curr_count"] - u["prev_count"]) * w["explore_bonus_weight"]
            return 0

        if self.kind == abi.WRAP_START_KIT:
            heal = 0
            if w["heal_bonus_weight"] > 0 and self._ent(st, e, a, "alive"):
                if self._ent(st, e, a, "health_restore") > 0:
                    heal = w["heal_bonus_weight"]
            reward += heal + explore()
        elif self.kind == abi.WRAP_TAKERU:
            if not done:
                reward += explore()
        elif self.kind == abi.WRAP_YAOFENG:
            if not done:
                d = self.data[e][a]
                hp = self._ent(st, e, a, "health")
                hp_bonus = (hp - d["hp"]) * w["hp_bonus_weight"]
                d["hp"] = hp
                exp = max(self._ent(st, e, a, s + "_exp") for s in SKILLS)
                exp_bonus = (exp - d["exp"]) * w["exp_bonus_weight"]
                d["exp"] = exp
                D = 0
                if "Item" in self.envs.config.systems:
                    for w0, _ in st["items"][e][a - 1]:
                        t, lvl, eq = int(w0) & 31, (int(w0) >> 5) & 15, (int(w0) >> 9) & 1
                        if t and eq:
                            D += 3 * lvl if 2 <= t <= 4 else 2 * lvl if 8 <= t <= 12 else 0
                defense = (D + D + D) / (15 * 3)
                defense_bonus = w["defense_bonus_weight"] * defense
                inflicted = int(np.sum(self.log[e][(self.log[e][:, COL["ent_id"]] == a)
                                                   & (self.log[e][:, COL["event"]] == EC.SCORE_HIT),
                                                   COL["damage"]]))
                attack_bonus = (inflicted - d["damage_inflicted"]) * w["attack_bonus_weight"]
                d["damage_inflicted"] = inflicted
                gold = self._ent(st, e, a, "gold")
                gold_bonus = (gold - d["gold"]) * w["gold_bonus_weight"]
                d["gold"] = gold
                reward += (hp_bonus + exp_bonus + defense_bonus + attack_bonus + gold_bonus) * w["custom_bonus_scale"]
        return reward

    def _observation(self, e, st, mask):
        obs = self.envs.obs
        if obs is None:
            return
        L = self.lay
        for a in self.ids:
            if not mask[a - 1] or not self._ent(st, e, a, "alive"):
                continue  # absent / dead agents carry an all-zero obs row
            row = obs[e, a - 1]
            at = {k.split(".", 1)[1]: s for k, s in L.items() if k.startswith("ActionTargets.")}

            def seg(name):
                s = at[name]
                return row[s.offset:s.offset + s.shape[0]]

            if self.kind == abi.WRAP_START_KIT:
                seg("Sell.Price")[self.hist[e][a]["prev_price"]] = 0
            if self.w.get("disable_give"):
                seg("Give.InventoryItem")[:-1] = 0
                seg("Give.Target")[:-1] = 0
                seg("GiveGold.Target")[:-1] = 0
                seg("GiveGold.Price")[1:] = 0
            if self.w.get("donot_attack_dangerous_npc"):
                ent = row[L["Entity"].offset:L["Entity"].offset + 100 * 31].reshape(100, 31)
                seg("Attack.Target")[np.where(ent[:, 1] > 1)] = 0
