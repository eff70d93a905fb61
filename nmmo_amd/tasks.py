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
