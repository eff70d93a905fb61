"""Task programs (SPEC.md §12) built the way the reference's curricula write them:
`task("CountEvent", event="EAT_FOOD", N=3)` mirrors `TaskSpec(eval_fn=CountEvent,
eval_fn_kwargs={"event": "EAT_FOOD", "N": 3})` (curriculum_generation/manual_curriculum.py:53-314,
neurips23_evaluation/heldout_evaluation_task.py:30-138). Agent tasks only: the subject is the
player itself, so `num_agent` must be 1 where a predicate takes it.
"""

from __future__ import annotations

from . import abi

EVENT = {k: v for k, v in vars(abi.EventCode).items() if k.isupper()}
ITEM = {"Hat": 2, "Top": 3, "Bottom": 4, "Spear": 5, "Bow": 6, "Wand": 7, "Rod": 8, "Gloves": 9,
        "Pickaxe": 10, "Axe": 11, "Chisel": 12, "Whetstone": 13, "Arrow": 14, "Runes": 15,
        "Ration": 16, "Potion": 17}
SKILL = {"Melee": 1, "Range": 2, "Mage": 3, "Fishing": 4, "Herbalism": 5, "Prospecting": 6,
         "Carving": 7, "Alchemy": 8}
MATERIAL = {"Void": 0, "Water": 1, "Grass": 2, "Scrub": 3, "Foilage": 4, "Stone": 5, "Slag": 6,
            "Ore": 7, "Stump": 8, "Tree": 9, "Fragment": 10, "Crystal": 11, "Weeds": 12, "Herb": 13,
            "Ocean": 14, "Fish": 15}
# manual_curriculum.py:42-51
TOOL_FOR_SKILL = {"Melee": "Spear", "Range": "Bow", "Mage": "Wand", "Fishing": "Rod",
                  "Herbalism": "Gloves", "Carving": "Axe", "Prospecting": "Pickaxe", "Alchemy": "Chisel"}


def _id(table, v):
    return v if isinstance(v, int) else table[v]


# SPEC §12 teams (nmmo's TeamHelper for the agent-training game: every agent its own team, in id
# order): the left team of agent i is agent i - 1 (1 -> PLAYER_N), the right one i + 1, and a
# one-agent team's leader is that agent
TEAM_TARGET = {"left_team_leader": -1, "right_team_leader": -2, "left_team": -1, "right_team": -2}


def _target(eval_fn, v):
    if eval_fn == "CanSeeAgent" and isinstance(v, int) and v > 0:
        return v
    if eval_fn == "CanSeeGroup" and isinstance(v, (list, tuple)) and len(v) == 1 and int(v[0]) > 0:
        return int(v[0])
    key = v if isinstance(v, str) else None
    ok = key in TEAM_TARGET and key.endswith("_leader") == (eval_fn == "CanSeeAgent")
    if not ok:
        raise ValueError(f"{eval_fn}: target {v!r} (agent tasks: left/right team"
                         f"{'_leader' if eval_fn == 'CanSeeAgent' else ''} or a player id)")
    return TEAM_TARGET[key]


def _one(kw):
    if kw.pop("num_agent", 1) != 1:
        raise ValueError("agent tasks only: num_agent must be 1 (team tasks are out of scope)")


def term(eval_fn: str, weight: float = 1.0, **kw) -> abi.NmmoTaskTerm:
    """One predicate term; argument names follow nmmo.task.base_predicates."""
    kw = dict(kw)
    a = b = c = 0
    if eval_fn == "TickGE":
        a = kw.pop("num_tick")
    elif eval_fn == "CountEvent":
        a, b = _id(EVENT, kw.pop("event")), kw.pop("N")
    elif eval_fn == "ScoreHit":
        a, b = _id(SKILL, kw.pop("combat_style")), kw.pop("N")
    elif eval_fn in ("HarvestItem", "ConsumeItem", "ListItem", "BuyItem", "OwnItem"):
        a, b, c = _id(ITEM, kw.pop("item")), kw.pop("level"), kw.pop("quantity")
    elif eval_fn in ("EarnGold", "SpendGold", "MakeProfit", "HoardGold"):
        a = kw.pop("amount")
    elif eval_fn == "DefeatEntity":
        kind = kw.pop("agent_type")
        a, b, c = {"npc": 0, "player": 1}[kind], kw.pop("level"), kw.pop("num_agent", 1)
    elif eval_fn == "AttainSkill":
        _one(kw)
        a, b = _id(SKILL, kw.pop("skill")), kw.pop("level")
    elif eval_fn == "GainExperience":
        _one(kw)
        a, b = _id(SKILL, kw.pop("skill")), kw.pop("experience")
    elif eval_fn == "EquipItem":
        _one(kw)
        a, b = _id(ITEM, kw.pop("item")), kw.pop("level")
    elif eval_fn == "InventorySpaceGE":
        a = kw.pop("space")
    elif eval_fn == "OccupyTile":
        a, b = kw.pop("row"), kw.pop("col")
    elif eval_fn == "CanSeeTile":
        a = _id(MATERIAL, kw.pop("tile_type"))
    elif eval_fn == "FullyArmed":
        _one(kw)
        a, b = _id(SKILL, kw.pop("combat_style")), kw.pop("level")
    elif eval_fn == "PracticeEating":  # curriculum_tutorial.py:45-57 (no arguments)
        pass
    elif eval_fn in ("CanSeeAgent", "CanSeeGroup"):  # manual_curriculum.py:157-162
        a = _target(eval_fn, kw.pop("target"))
    else:
        raise ValueError(f"unsupported predicate {eval_fn!r}")
    if kw:
        raise TypeError(f"{eval_fn}: unexpected arguments {sorted(kw)}")
    return abi.NmmoTaskTerm(abi.PRED[eval_fn], int(a), int(b), int(c), float(weight), 0)


def task(eval_fn: str, **kw) -> abi.NmmoTask:
    t = abi.NmmoTask()
    t.term[0] = term(eval_fn, **kw)
    t.combine = abi.TASK_SINGLE
    return t


def practice_skill_with_tool(skill: str, exp: int) -> abi.NmmoTask:
    """manual_curriculum.py:113-117: 0.3 * EquipItem(tool, level 1) + 0.7 * GainExperience."""
    t = abi.NmmoTask()
    t.term[0] = term("EquipItem", weight=0.3, item=TOOL_FOR_SKILL[skill], level=1)
    t.term[1] = term("GainExperience", weight=0.7, skill=skill, experience=exp)
    t.combine = abi.TASK_SUM
    return t


def practice_inventory_management(space: int, num_tick: int) -> abi.NmmoTask:
    """manual_curriculum.py:203-204: InventorySpaceGE(space) * TickGE(num_tick)."""
    t = abi.NmmoTask()
    t.term[0] = term("InventorySpaceGE", space=space)
    t.term[1] = term("TickGE", num_tick=num_tick)
    t.combine = abi.TASK_PRODUCT
    return t


def practice_eating() -> abi.NmmoTask:
    """curriculum_tutorial.py:45-57: progress = 0.06 per EAT_FOOD, +0.1 at the 1st, +0.3 at the 3rd."""
    return task("PracticeEating")


# custom eval functions of the reference's curricula: name -> builder(**eval_fn_kwargs)
COMPOSITES = {
    "PracticeSkillWithTool": lambda skill, exp: practice_skill_with_tool(skill, exp),
    "PracticeInventoryManagement": lambda space, num_tick: practice_inventory_management(space, num_tick),
    "PracticeEating": lambda: practice_eating(),
}


def _kw_str(v) -> str:
    return v if isinstance(v, str) else str(v)


def spec_name(eval_fn: str, reward_to: str = "agent", **kw) -> str:
    """nmmo TaskSpec.name: "Task_<eval_fn>_(<k>:<v>_...)_reward_to:<reward_to>", kwargs in
    insertion order, classes by name (pinned by the reference's heldout task names,
    tests/golden/task_embeddings.npz heldout_names)."""
    args = "(" + "".join(f"{k}:{_kw_str(v)}_" for k, v in kw.items())[:-1] + ")"
    return "_".join(["Task", eval_fn, args, "reward_to:" + reward_to])


class TaskSpec:
    """nmmo.task.task_spec.TaskSpec for agent tasks: eval_fn (a base predicate or one of the
    curricula's custom functions, by name; items/skills/materials by name), eval_fn_kwargs,
    sampling_weight (curriculum sampling, manual_curriculum.py) and an optional fp16 embedding
    (the Task obs; the reference's *_with_embedding.pkl)."""

    def __init__(self, eval_fn: str, eval_fn_kwargs: dict | None = None, sampling_weight: float = 1.0,
                 embedding=None, reward_to: str = "agent"):
        if reward_to != "agent":
            raise ValueError("agent tasks only (team tasks are out of scope)")
        self.eval_fn = eval_fn
        self.eval_fn_kwargs = dict(eval_fn_kwargs or {})
        self.sampling_weight = sampling_weight
        self.embedding = embedding
        self.reward_to = reward_to

    @property
    def name(self) -> str:
        return spec_name(self.eval_fn, self.reward_to, **self.eval_fn_kwargs)

    def program(self) -> abi.NmmoTask:
        if self.eval_fn in COMPOSITES:
            return COMPOSITES[self.eval_fn](**self.eval_fn_kwargs)
        return task(self.eval_fn, **self.eval_fn_kwargs)

    def __repr__(self):
        return f"TaskSpec({self.name}, w={self.sampling_weight})"


# nmmo.systems.skill / item groupings the curricula iterate (order as nmmo defines them)
COMBAT_SKILL = ["Melee", "Range", "Mage"]
HARVEST_SKILL = ["Fishing", "Herbalism", "Prospecting", "Carving", "Alchemy"]
ARMOR = ["Hat", "Top", "Bottom"]
WEAPON = ["Spear", "Bow", "Wand"]
TOOL = ["Rod", "Gloves", "Pickaxe", "Axe", "Chisel"]
AMMUNITION = ["Whetstone", "Arrow", "Runes"]
CONSUMABLE = ["Ration", "Potion"]
ALL_ITEM = ARMOR + WEAPON + TOOL + AMMUNITION + CONSUMABLE
HARVESTABLE = ["Water", "Foilage", "Ore", "Tree", "Crystal", "Herb", "Fish"]  # nmmo.lib.material


def heldout_curriculum() -> list:
    """The 63 held-out evaluation tasks, neurips23_evaluation/heldout_evaluation_task.py:30-138."""
    event_goal, level_goal, gold_goal = 20, [1, 3], 100
    c = [TaskSpec("TickGE", {"num_tick": 1024}),
         TaskSpec("CountEvent", {"event": "PLAYER_KILL", "N": event_goal})]
    c += [TaskSpec("DefeatEntity", {"agent_type": "npc", "level": lv, "num_agent": event_goal}) for lv in level_goal]
    c += [TaskSpec("CountEvent", {"event": "GO_FARTHEST", "N": 64}),
          TaskSpec("OccupyTile", {"row": 80, "col": 80})]
    c += [TaskSpec("AttainSkill", {"skill": sk, "level": 10, "num_agent": 1}) for sk in COMBAT_SKILL + HARVEST_SKILL]
    c += [TaskSpec("HarvestItem", {"item": it, "level": lv, "quantity": event_goal})
          for it in AMMUNITION for lv in level_goal]
    c += [TaskSpec("ConsumeItem", {"item": it, "level": lv, "quantity": event_goal})
          for it in CONSUMABLE for lv in level_goal]
    c += [TaskSpec("EquipItem", {"item": it, "level": lv, "num_agent": 1})
          for it in ARMOR + WEAPON + TOOL + AMMUNITION for lv in level_goal]
    c += [TaskSpec("FullyArmed", {"combat_style": sk, "level": lv, "num_agent": 1})
          for sk in COMBAT_SKILL for lv in level_goal]
    c += [TaskSpec("CountEvent", {"event": "EARN_GOLD", "N": event_goal}),
          TaskSpec("CountEvent", {"event": "BUY_ITEM", "N": event_goal}),
          TaskSpec("EarnGold", {"amount": gold_goal}),
          TaskSpec("HoardGold", {"amount": gold_goal}),
          TaskSpec("MakeProfit", {"amount": gold_goal})]
    return c


def manual_curriculum() -> list:
    """curriculum_generation/manual_curriculum.py:53-314, every spec of the file in its order,
    with their sampling weights (CanSeeAgent / CanSeeGroup at :157-162 target the neighbouring
    teams, SPEC §12)."""
    event_goal = [1, 2, 3, 5, 7, 9, 12, 15, 20, 30, 50]
    infrequent, stay_alive = list(range(1, 10)), [50, 100, 150, 200, 300, 500, 700]
    level_goal, item_num = list(range(2, 10)), [1, 2, 3, 4, 5]
    c = [TaskSpec("TickGE", {"num_tick": 1024})]
    c += [TaskSpec("CountEvent", {"event": ev, "N": n}, sampling_weight=100)
          for ev in ["EAT_FOOD", "DRINK_WATER"] for n in range(1, 10)]
    c += [TaskSpec("CountEvent", {"event": ev, "N": n}, sampling_weight=20)
          for ev in ["SCORE_HIT", "PLAYER_KILL", "HARVEST_ITEM", "EQUIP_ITEM", "CONSUME_ITEM", "LEVEL_UP",
                     "EARN_GOLD", "LIST_ITEM", "BUY_ITEM"] for n in event_goal]
    c += [TaskSpec("CountEvent", {"event": ev, "N": n})
          for ev in ["GIVE_ITEM", "DESTROY_ITEM", "GIVE_GOLD"] for n in infrequent]
    c += [TaskSpec("CanSeeTile", {"tile_type": m}, sampling_weight=10) for m in HARVESTABLE]
    for sk in COMBAT_SKILL + HARVEST_SKILL:
        c += [TaskSpec("AttainSkill", {"skill": sk, "level": lv, "num_agent": 1},
                       sampling_weight=10 * (6 - lv) if lv < 6 else 5) for lv in level_goal[1:]]
        c += [TaskSpec("PracticeSkillWithTool", {"skill": sk, "exp": e}, sampling_weight=50) for e in stay_alive]
    c += [TaskSpec("TickGE", {"num_tick": n}) for n in stay_alive]
    c += [TaskSpec("OccupyTile", {"row": 80, "col": 80})]
    c += [TaskSpec("CanSeeAgent", {"target": t}) for t in ["left_team_leader", "right_team_leader"]]
    c += [TaskSpec("CanSeeGroup", {"target": t}) for t in ["left_team", "right_team"]]
    c += [TaskSpec("ScoreHit", {"combat_style": st, "N": n}, sampling_weight=5)
          for st in COMBAT_SKILL for n in event_goal]
    for fn, w in [("HoardGold", 10), ("EarnGold", 10), ("SpendGold", 5), ("MakeProfit", 3)]:
        c += [TaskSpec(fn, {"amount": a}, sampling_weight=w) for a in event_goal]
    c += [TaskSpec("PracticeInventoryManagement", {"space": sp, "num_tick": n})
          for sp in [2, 4, 8] for n in stay_alive]

    def item_tasks(fn, items):
        return [TaskSpec(fn, {"item": it, "level": lv, "quantity": q}, sampling_weight=4 - lv if lv < 4 else 1)
                for it in items for lv in level_goal for q in item_num if lv + q <= 6 or q == 1]

    c += item_tasks("OwnItem", ALL_ITEM)
    c += [TaskSpec("EquipItem", {"item": it, "level": lv, "num_agent": 1}, sampling_weight=4 - lv if lv < 4 else 1)
          for it in ARMOR + WEAPON + TOOL + AMMUNITION for lv in level_goal]
    c += item_tasks("ConsumeItem", CONSUMABLE)
    c += item_tasks("HarvestItem", WEAPON + AMMUNITION + CONSUMABLE)
    c += item_tasks("ListItem", ALL_ITEM)
    c += item_tasks("BuyItem", ALL_ITEM)
    return c


def tutorial_curriculum() -> list:
    """curriculum_generation/curriculum_tutorial.py:22-72."""
    c = [TaskSpec("CountEvent", {"event": ev, "N": 10})
         for ev in ["GO_FARTHEST", "EAT_FOOD", "DRINK_WATER", "SCORE_HIT", "HARVEST_ITEM", "LEVEL_UP"]]
    c.append(TaskSpec("PracticeEating", {}))
    c += [TaskSpec("PracticeInventoryManagement", {"space": sp, "num_tick": 500}) for sp in [2, 4, 8]]
    return c


def sample_eval_curriculum() -> list:
    """The 24 sample evaluation tasks, neurips23_evaluation/sample_evaluation_task.py:12-52
    (sample_eval_task_with_embedding.pkl holds their embeddings in this order)."""
    c = [TaskSpec("TickGE", {"num_tick": 1024})]
    c += [TaskSpec("CountEvent", {"event": ev, "N": 10})
          for ev in ["EAT_FOOD", "DRINK_WATER", "SCORE_HIT", "PLAYER_KILL", "HARVEST_ITEM", "EQUIP_ITEM",
                     "CONSUME_ITEM", "LEVEL_UP", "EARN_GOLD", "LIST_ITEM", "BUY_ITEM", "GIVE_ITEM",
                     "DESTROY_ITEM", "GIVE_GOLD"]]
    c += [TaskSpec("AttainSkill", {"skill": sk, "level": 10, "num_agent": 1}) for sk in COMBAT_SKILL + HARVEST_SKILL]
    c += [TaskSpec("EarnGold", {"amount": 50})]
    return c
