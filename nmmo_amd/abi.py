"""ctypes mirror of include/nmmo_hip.h (the C-ABI boundary).

Field enums and struct layouts must match the header exactly; tests/test_abi.py checks the
struct sizes against the compiled library and the enum values against the header text.
"""

import ctypes

ABI_VERSION = 8

NMMO_OK = 0
NMMO_E_INVALID = -1
NMMO_E_HIP = -2
NMMO_E_NOMEM = -3
NMMO_E_SIZE = -4

# tick fault word (nmmo_get_fault): code | env << 8
FAULT_ATTACK_ROUNDS = 1
FAULT_BUY_ROUNDS = 2
FAULT_GIVE_ROUNDS = 3
FAULT_HASH_PROBE = 4
FAULT_ENV_LIST = 5
FAULT_WIRE_SCAN = 6
FAULT_NAMES = {1: "attack rounds", 2: "Buy rounds", 3: "Give rounds", 4: "position-hash probe",
               5: "env id outside the handle (nmmo_step_envs)", 6: "wire payload offset scan"}

SYS_RESOURCE = 1 << 0
SYS_COMBAT = 1 << 1
SYS_NPC = 1 << 2
SYS_PROGRESSION = 1 << 3
SYS_ITEM = 1 << 4
SYS_EQUIPMENT = 1 << 5
SYS_PROFESSION = 1 << 6
SYS_EXCHANGE = 1 << 7
SYS_ALL = 0xFF

OBS_NONE = 0
OBS_FLAT = 1
OBS_NATIVE = 2
OBS_SEC_TILE = 1  # nmmo_obs_invalidate_sections: the Tile section
OBS_SEC_ALL = 0xFFFFFFFF
STORE_CTL_INTS = 16  # nmmo_exp_store_records_checked's device words (per-input check bits)
OBS_WIRE = 3  # SPEC.md §8c wire records straight from the state (the learner-gather transport)
# native layout (SPEC.md §8b)
NATIVE_MASK_BYTES = 1600
NATIVE_I16 = 3976
NATIVE_ROW_BYTES = NATIVE_MASK_BYTES + 2 * NATIVE_I16
NATIVE_MARKET_BYTES = 1024 * 16 * 2


def native_env_bytes(players: int = 128) -> int:
    return players * NATIVE_ROW_BYTES + NATIVE_MARKET_BYTES

MAP_SIZE = 160
MAP_TILES = MAP_SIZE * MAP_SIZE
N_ENTITY_COLS = 31
N_ACTION_HEADS = 12
NF = 48
NE = 16

# Entity table fields (int16 [n_envs][NF][slots]); 0..30 are the Entity obs columns.
ENTITY_FIELDS = [
    "id", "npc_type", "row", "col", "damage", "time_alive", "freeze", "item_level",
    "attacker_id", "latest_combat_tick", "message", "gold", "health", "food", "water",
    "melee_level", "melee_exp", "range_level", "range_exp", "mage_level", "mage_exp",
    "fishing_level", "fishing_exp", "herbalism_level", "herbalism_exp",
    "prospecting_level", "prospecting_exp", "carving_level", "carving_exp",
    "alchemy_level", "alchemy_exp",
    # internal
    "alive", "ds_row", "resilient", "exploration", "style", "target_id", "npc_level",
    "equip_offense", "equip_defense", "player_kills", "health_restore", "died_tick",
    "drop_armor", "drop_tool",
]
F = {name: i for i, name in enumerate(ENTITY_FIELDS)}

ENV_FIELDS = [
    "tick", "map_id", "done", "episode", "npc_count", "npc_next_id", "free_head",
    "free_count", "seed_lo", "seed_hi", "players_alive", "env_index",
    "item_free_head", "item_free_count", "event_count",
]
E = {name: i for i, name in enumerate(ENV_FIELDS)}

# Event log (SPEC.md §11): int32 rows of EVENT_ATTRS; nmmo's column aliases (ATTR_TO_COL) as read
# by the reference (stat_wrapper.py:219-300).
EVENT_COLS = 9
EVENT_ATTRS = ["id", "ent_id", "tick", "event", "type", "level", "number", "gold", "target_ent"]
ATTR_TO_COL = {a: i for i, a in enumerate(EVENT_ATTRS)}
ATTR_TO_COL.update(item_type=4, combat_style=4, quantity=6, damage=6, distance=6, price=7)


# Tasks (SPEC.md §12)
PREDICATES = [
    "NONE", "TickGE", "CountEvent", "ScoreHit", "HarvestItem", "ConsumeItem", "ListItem", "BuyItem",
    "EarnGold", "SpendGold", "MakeProfit", "DefeatEntity", "HoardGold", "AttainSkill",
    "GainExperience", "EquipItem", "OwnItem", "InventorySpaceGE", "OccupyTile", "CanSeeTile",
    "FullyArmed", "PracticeEating", "CanSeeAgent", "CanSeeGroup",
]
PRED = {n: i for i, n in enumerate(PREDICATES)}
TASK_SINGLE, TASK_SUM, TASK_PRODUCT = 0, 1, 2
MAX_TASKS = 4096


class NmmoTaskTerm(ctypes.Structure):
    _fields_ = [("pred", ctypes.c_int32), ("a", ctypes.c_int32), ("b", ctypes.c_int32),
                ("c", ctypes.c_int32), ("weight", ctypes.c_float), ("reserved", ctypes.c_int32)]


class NmmoTask(ctypes.Structure):
    _fields_ = [("term", NmmoTaskTerm * 2), ("combine", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class NmmoTaskState(ctypes.Structure):
    _fields_ = [("last", ctypes.c_double), ("max_progress", ctypes.c_double),
                ("acc", ctypes.c_int32 * 4), ("signals", ctypes.c_int32),
                ("completed_tick", ctypes.c_int32)]


def task_state_dtype():
    import numpy as np

    return np.dtype([("last", "<f8"), ("max_progress", "<f8"), ("acc", "<i4", (4,)),
                     ("signals", "<i4"), ("completed_tick", "<i4")])


class EventCode:
    """nmmo.lib.event_code.EventCode (nmmo 2.1, SPEC.md §11)."""
    EAT_FOOD = 1
    DRINK_WATER = 2
    GO_FARTHEST = 3
    SCORE_HIT = 11
    PLAYER_KILL = 12
    CONSUME_ITEM = 21
    GIVE_ITEM = 22
    DESTROY_ITEM = 23
    HARVEST_ITEM = 24
    EQUIP_ITEM = 25
    LOOT_ITEM = 26
    GIVE_GOLD = 31
    LIST_ITEM = 32
    EARN_GOLD = 33
    BUY_ITEM = 34
    LEVEL_UP = 41
    AGENT_CULLED = 91


class NmmoConfig(ctypes.Structure):
    _fields_ = [
        ("abi_version", ctypes.c_int32),
        ("player_n", ctypes.c_int32),
        ("npc_n", ctypes.c_int32),
        ("horizon", ctypes.c_int32),
        ("map_n", ctypes.c_int32),
        ("spawn_immunity", ctypes.c_int32),
        ("early_stop_agent_num", ctypes.c_int32),
        ("resilient_u32", ctypes.c_uint32),
        ("systems", ctypes.c_uint32),
        ("obs_layout", ctypes.c_int32),
        ("task_embed_dim", ctypes.c_int32),
        ("task_num_tick", ctypes.c_int32),
        ("event_cap", ctypes.c_int32),
        ("reserved0", ctypes.c_int32),
        ("map_seed", ctypes.c_uint64),
        ("env_index_base", ctypes.c_uint64),
    ]


_MASK_NAMES = [
    "mask_attack_style", "mask_attack_target", "mask_buy", "mask_destroy", "mask_give_item",
    "mask_give_target", "mask_givegold_price", "mask_givegold_target", "mask_move",
    "mask_sell_item", "mask_sell_price", "mask_use",
]


class NmmoLayout(ctypes.Structure):
    _fields_ = (
        [("obs_elems", ctypes.c_int32), ("act_heads", ctypes.c_int32),
         ("act_dims", ctypes.c_int32 * N_ACTION_HEADS)]
        + [("off_" + n, ctypes.c_int32) for n in _MASK_NAMES]
        + [("off_" + n, ctypes.c_int32) for n in
           ["agent_id", "current_tick", "entity", "inventory", "market", "task", "tile"]]
        + [(n, ctypes.c_int32) for n in
           ["entity_rows", "entity_cols", "inventory_rows", "item_cols", "market_rows",
            "tile_rows", "tile_cols", "slots", "nf", "ne"]]
        + [("state_bytes_per_env", ctypes.c_size_t)]
    )


INV_SLOTS = 12
MARKET_ROWS = 1024


TASK_STATE_BYTES = 40


def state_bytes_per_env(slots: int, players: int = 128) -> int:
    return NE * 4 + NF * slots * 2 + slots * 2 + MAP_TILES + players * INV_SLOTS * 8 \
        + INV_SLOTS * players * 2 + players * 4 + players * TASK_STATE_BYTES


# Wrapper layer (SPEC.md §13; nmmo_set_wrapper)
WRAP_BASE, WRAP_START_KIT, WRAP_TAKERU, WRAP_YAOFENG = 0, 1, 2, 3
UNIQ_WORDS = 153
# NmmoAgentInfo.performed bit order (stat_wrapper.py:196-205 KEY_EVENT, then :207-236)
PERFORMED_KEYS = ["eat_food", "drink_water", "score_hit", "player_kill", "consume_item",
                  "harvest_item", "list_item", "buy_item", "equip_armor", "equip_weapon",
                  "equip_tool", "equip_ammo", "harvest_weapon"]
ITEM_CATEGORIES = ["armor", "weapon", "tool", "ammo", "consumable"]


class NmmoWrapperConfig(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("use_custom_reward", ctypes.c_int32),
                ("eval_mode", ctypes.c_int32), ("clip_unique_event", ctypes.c_int32),
                ("disable_give", ctypes.c_int32), ("donot_attack_dangerous_npc", ctypes.c_int32),
                ("heal_bonus_weight", ctypes.c_double), ("explore_bonus_weight", ctypes.c_double),
                ("hp_bonus_weight", ctypes.c_double), ("exp_bonus_weight", ctypes.c_double),
                ("defense_bonus_weight", ctypes.c_double), ("attack_bonus_weight", ctypes.c_double),
                ("gold_bonus_weight", ctypes.c_double), ("custom_bonus_scale", ctypes.c_double)]


def agent_info_dtype():
    import numpy as np

    return np.dtype([("done", "<i4"), ("length", "<i4"), ("ret", "<f8"), ("max_progress", "<f8"),
                     ("reward_signal_count", "<i4"), ("task_completed", "<i4"),
                     ("cod_attacked", "<i4"), ("cod_starved", "<i4"), ("cod_dehydrated", "<i4"),
                     ("max_combat_level", "<i4"), ("max_harvest_skill_ammo", "<i4"),
                     ("max_harvest_skill_consum", "<i4"), ("performed", "<u4"),
                     ("max_progress_to_center", "<i4"), ("earned_gold", "<i4"), ("max_damage", "<i4"),
                     ("max_item_level", "<i4", (5,)), ("agent_kill_count", "<i4"),
                     ("npc_kill_count", "<i4"), ("unique_events", "<i4")])


def wrap_state_dtype():
    import numpy as np

    return np.dtype([("cum_reward", "<f8"), ("prev_count", "<i4"), ("curr_count", "<i4"),
                     ("prev_price", "<i4"), ("hp", "<i4"), ("exp", "<i4"), ("gold", "<i4"),
                     ("dmg_inflicted_prev", "<i4"), ("dmg_inflicted", "<i4"), ("performed", "<u4"),
                     ("max_dist", "<i4"), ("earned_gold", "<i4"), ("max_damage", "<i4"),
                     ("max_item_level", "<i4", (5,)), ("agent_kills", "<i4"), ("npc_kills", "<i4"),
                     ("reserved", "<i4")])


# ---------------------------------------------------------------- experience storage
class NmmoExperience(ctypes.Structure):
    _fields_ = [("capacity", ctypes.c_int32), ("obs_elems", ctypes.c_int32), ("n_slots", ctypes.c_int32)] + [
        (n, ctypes.c_void_p) for n in ("obs", "actions", "logprobs", "rewards", "dones", "truncateds", "values",
                                       "env_id", "step", "seq", "slot_count", "ptr", "status")]


class NmmoRecordStore(ctypes.Structure):
    """Compact experience observations (nmmo_exp_store_records / nmmo_exp_gather_records)."""
    _fields_ = [("arena", ctypes.c_void_p), ("arena_bytes", ctypes.c_int64), ("arena_used", ctypes.c_void_p),
                ("row_buf", ctypes.c_void_p), ("row_agent", ctypes.c_void_p)]


P2P_ID_BYTES = 128  # nmmo_p2p_unique_id


class NmmoP2POp(ctypes.Structure):
    _fields_ = [("buf", ctypes.c_void_p), ("bytes", ctypes.c_int64), ("peer", ctypes.c_int32), ("recv", ctypes.c_int32)]


class NmmoStoreInput(ctypes.Structure):
    _fields_ = [("n_rows", ctypes.c_int32), ("step", ctypes.c_int32), ("obs", ctypes.c_void_p),
                ("native", ctypes.c_void_p), ("rewards", ctypes.c_void_p), ("dones", ctypes.c_void_p),
                ("mask", ctypes.c_void_p), ("env_id", ctypes.c_void_p), ("env_id_base", ctypes.c_int32),
                ("actions", ctypes.c_void_p), ("logprobs", ctypes.c_void_p), ("values", ctypes.c_void_p),
                ("wire", ctypes.c_void_p)]
