/*
 * nmmo_hip.h — C-ABI of the MI355X-native Neural MMO env stepper (libnmmo_hip.so).
 *
 * This is the drop-in boundary for the reference's hot path. The reference (Meeso1/nmmo,
 * NeurIPS-2023 baselines) reaches the simulator only through Python protocols — there is no
 * FFI in the reference to bind against — so each entry point below names the reference call
 * site whose behaviour it replaces:
 *
 *   nmmo_create   <- nmmo.Env(Config(...))            reinforcement_learning/environment.py:57
 *                    + pufferlib pool construction     reinforcement_learning/clean_pufferl.py:106-114
 *   nmmo_reset    <- pool.async_reset(seed)            clean_pufferl.py:175
 *                    -> env.reset(seed=...)            reinforcement_learning/stat_wrapper.py:51
 *   nmmo_step     <- pool.send(actions); pool.recv()   clean_pufferl.py:357, :293
 *                    -> env.step(actions)              stat_wrapper.py:64
 *   nmmo_layout   <- pool.single_observation_space / driver_env.unflatten_context
 *                                                      clean_pufferl.py:116, baseline_policy.py:28,41
 *   nmmo_get_state / nmmo_set_state  <- env.realm.{players,npcs,map,tick} reads
 *                                                      stat_wrapper.py:122-185, train_helper.py:133-166
 *   nmmo_set_wrapper <- env_creator's RewardWrapper(BaseStatWrapper) around each env
 *                    (reward shaping, obs edits, info) environment.py:58, stat_wrapper.py:57-185
 *   nmmo_scripted_actions  <- (bench/test helper) masked-uniform actions, the behaviour of an
 *                    untrained masked policy           agent_zoo/neurips23_start_kit/baseline_policy.py:228-264
 *
 * Conventions: every call returns 0 on success or a negative NMMO_E_* code (never aborts);
 * nmmo_last_error() returns a thread-local message. Every I/O buffer passed to step/reset is a
 * caller-owned DEVICE pointer (e.g. torch tensor .data_ptr()); the handle owns the env state in
 * HBM. Work is enqueued on `stream` (a hipStream_t, NULL = default stream) with no implicit
 * device synchronisation and no allocation inside step (graph-capturable). One host thread per
 * handle; handles are independent (one per GPU rank).
 *
 * The game semantics these calls implement are frozen in SPEC.md (v1); the state layout below
 * is shared bit-for-bit with the CPU oracle under oracle/ (test infrastructure only).
 */
#ifndef NMMO_HIP_H
#define NMMO_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NMMO_API __attribute__((visibility("default")))
#define NMMO_ABI_VERSION 8

/* ---- error codes ---- */
#define NMMO_OK 0
#define NMMO_E_INVALID (-1)   /* bad argument / config */
#define NMMO_E_HIP (-2)       /* HIP runtime error */
#define NMMO_E_NOMEM (-3)     /* device allocation failed */
#define NMMO_E_SIZE (-4)      /* buffer size mismatch */

/* ---- systems bitmask (mirrors the Config mixins, environment.py:14-25) ---- */
#define NMMO_SYS_RESOURCE (1u << 0)
#define NMMO_SYS_COMBAT (1u << 1)
#define NMMO_SYS_NPC (1u << 2)
#define NMMO_SYS_PROGRESSION (1u << 3)
#define NMMO_SYS_ITEM (1u << 4)
#define NMMO_SYS_EQUIPMENT (1u << 5)
#define NMMO_SYS_PROFESSION (1u << 6)
#define NMMO_SYS_EXCHANGE (1u << 7)
#define NMMO_SYS_ALL 0xFFu

/* ---- observation layouts ---- */
#define NMMO_OBS_NONE 0   /* C2/C3 benchmark configs: state only */
#define NMMO_OBS_FLAT 1   /* pufferlib-0.7.3 flat float32 vector, 23,987 / agent */
#define NMMO_OBS_NATIVE 2 /* nmmo space dtypes, Market once per env (SPEC.md §8b) */
#define NMMO_OBS_WIRE 3   /* the wire records of SPEC.md §8c written straight from the state
                             (the learner-gather transport; nmmo_wire_unpack gives the native
                             layout, nmmo_exp_store decodes kept rows to flat rows) */
#define NMMO_NATIVE_MASK_BYTES 1600   /* u8 ActionTargets (1,586) + pad */
#define NMMO_NATIVE_I16 3976          /* int16 part of an agent row */
#define NMMO_NATIVE_ROW_BYTES (NMMO_NATIVE_MASK_BYTES + 2 * NMMO_NATIVE_I16)  /* 9,552 */
#define NMMO_NATIVE_MARKET_BYTES (NMMO_MARKET_ROWS * 16 * 2)               /* 32,768 per env */

/* ---- items (SPEC.md §9): per player NMMO_INV_SLOTS inventory slots in ascending item-row
 * order, each item two u32 words: w0 = type | level<<5 | equipped<<9 | listed_price<<10 |
 * listed_tick<<17 ; w1 = quantity | row<<16 (type 0 = empty slot). Item rows come from a FIFO
 * ring of NMMO_INV_SLOTS * player_n rows. ---- */
#define NMMO_INV_SLOTS 12
#define NMMO_MARKET_ROWS 1024

/* ---- fixed geometry (nmmo 2.1 defaults, SPEC.md §1) ---- */
#define NMMO_MAP_SIZE 160          /* MAP_CENTER 128 + 2 * MAP_BORDER 16 */
#define NMMO_MAP_TILES (NMMO_MAP_SIZE * NMMO_MAP_SIZE)
#define NMMO_N_MATERIALS 16
#define NMMO_N_ENTITY_COLS 31      /* Entity obs columns (baseline_policy.py:118) */
#define NMMO_N_ACTION_HEADS 12     /* takeru/policy.py:293-307 */

/* Entity table fields: int16 [n_envs][NMMO_NF][slots]; fields 0..30 ARE the Entity obs
 * columns, in nmmo EntityState order (id col 0, npc_type col 1: baseline_policy.py:118-129). */
enum NmmoField {
  F_ID = 0, F_NPC_TYPE, F_ROW, F_COL, F_DAMAGE, F_TIME_ALIVE, F_FREEZE, F_ITEM_LEVEL,
  F_ATTACKER_ID, F_LATEST_COMBAT_TICK, F_MESSAGE, F_GOLD, F_HEALTH, F_FOOD, F_WATER,
  F_MELEE_LEVEL, F_MELEE_EXP, F_RANGE_LEVEL, F_RANGE_EXP, F_MAGE_LEVEL, F_MAGE_EXP,
  F_FISHING_LEVEL, F_FISHING_EXP, F_HERBALISM_LEVEL, F_HERBALISM_EXP,
  F_PROSPECTING_LEVEL, F_PROSPECTING_EXP, F_CARVING_LEVEL, F_CARVING_EXP,
  F_ALCHEMY_LEVEL, F_ALCHEMY_EXP,
  /* --- internal (not observed) --- */
  F_ALIVE = 31,        /* 1 while in the realm */
  F_DS_ROW,            /* datastore row (1-based; obs Entity rows are listed in this order) */
  F_RESILIENT,         /* RESOURCE_RESILIENT_POPULATION draw */
  F_EXPLORATION,       /* history.exploration (GO_FARTHEST record) */
  F_STYLE,             /* NPC combat style 0 melee 1 range 2 mage */
  F_TARGET_ID,         /* NPC AI target (player id, 0 = none) */
  F_NPC_LEVEL,         /* NPC spawn level */
  F_EQUIP_OFFENSE,     /* NPC equipment offense (equipment system) */
  F_EQUIP_DEFENSE,     /* NPC equipment defense */
  F_PLAYER_KILLS,
  F_HEALTH_RESTORE,    /* Resources.health_restore of the last update */
  F_DIED_TICK,         /* tick at which the player was culled (0 = alive) */
  F_DROP_ARMOR,        /* NPC drop: armor type - 2 (Hat/Top/Bottom) */
  F_DROP_TOOL,         /* NPC drop: tool type - 8 (Rod..Chisel) */
  NMMO_NF_USED,
  NMMO_NF = 48
};

/* Env scalar fields: int32 [n_envs][NMMO_NE]. */
enum NmmoEnvField {
  E_TICK = 0, E_MAP_ID, E_DONE, E_EPISODE, E_NPC_COUNT, E_NPC_NEXT_ID, E_FREE_HEAD,
  E_FREE_COUNT, E_SEED_LO, E_SEED_HI, E_PLAYERS_ALIVE, E_ENV_INDEX,
  E_ITEM_FREE_HEAD, E_ITEM_FREE_COUNT,
  E_EVENT_COUNT,       /* events logged in this episode (SPEC.md §11) */
  NMMO_NE_USED,
  NMMO_NE = 16
};

/* ---- event log (SPEC.md §11; nmmo.lib.event_log): per env a ring of event_cap rows of
 * NMMO_EVENT_COLS int32: id, ent_id, tick, event, type, level, number, gold, target_ent
 * (stat_wrapper.py:219-300 reads cols event/item_type/level/distance/gold/damage/target_ent). */
#define NMMO_EVENT_COLS 9
enum NmmoEventCode {
  EV_EAT_FOOD = 1, EV_DRINK_WATER = 2, EV_GO_FARTHEST = 3, EV_SCORE_HIT = 11, EV_PLAYER_KILL = 12,
  EV_CONSUME_ITEM = 21, EV_GIVE_ITEM = 22, EV_DESTROY_ITEM = 23, EV_HARVEST_ITEM = 24,
  EV_EQUIP_ITEM = 25, EV_LOOT_ITEM = 26, EV_GIVE_GOLD = 31, EV_LIST_ITEM = 32, EV_EARN_GOLD = 33,
  EV_BUY_ITEM = 34, EV_LEVEL_UP = 41, EV_AGENT_CULLED = 91
};

/* ---- tasks (SPEC.md §12; nmmo.task base predicates): a task program is up to two predicate
 * terms combined as SINGLE / SUM (w0*p0 + w1*p1) / PRODUCT (p0*p1); each player runs one. ---- */
enum NmmoPredicate {
  PRED_NONE = 0, PRED_TICK_GE = 1, PRED_COUNT_EVENT, PRED_SCORE_HIT, PRED_HARVEST_ITEM,
  PRED_CONSUME_ITEM, PRED_LIST_ITEM, PRED_BUY_ITEM, PRED_EARN_GOLD, PRED_SPEND_GOLD,
  PRED_MAKE_PROFIT, PRED_DEFEAT_ENTITY, PRED_HOARD_GOLD, PRED_ATTAIN_SKILL, PRED_GAIN_EXPERIENCE,
  PRED_EQUIP_ITEM, PRED_OWN_ITEM, PRED_INVENTORY_SPACE_GE, PRED_OCCUPY_TILE, PRED_CAN_SEE_TILE,
  PRED_FULLY_ARMED,
  PRED_PRACTICE_EATING, /* curriculum_generation/curriculum_tutorial.py:45-57 (EAT_FOOD count) */
  PRED_CAN_SEE_AGENT,   /* a = target agent id; -1 / -2: the left / right team's leader */
  PRED_CAN_SEE_GROUP,   /* a = -1 / -2: any member of the left / right team (SPEC.md §12 teams) */
  NMMO_N_PREDICATES
};
#define NMMO_TASK_SINGLE 0
#define NMMO_TASK_SUM 1
#define NMMO_TASK_PRODUCT 2
#define NMMO_MAX_TASKS 4096
typedef struct NmmoTaskTerm {
  int32_t pred;               /* NmmoPredicate */
  int32_t a, b, c;            /* predicate arguments, SPEC.md §12 table */
  float weight;               /* SUM weight */
  int32_t reserved;
} NmmoTaskTerm;
typedef struct NmmoTask {
  NmmoTaskTerm term[2];
  int32_t combine;            /* NMMO_TASK_* */
  int32_t reserved;
} NmmoTask;
/* per player task state (part of the state blob): previous / max progress, event accumulators,
 * positive-reward count (task.reward_signal_count), tick of first progress >= 1 (0 = none) */
typedef struct NmmoTaskState {
  double last, max_progress;
  int32_t acc[4];             /* term k uses acc[2k], acc[2k+1] */
  int32_t signals, completed_tick;
} NmmoTaskState;

/* ---- wrapper layer (SPEC.md §13): the reference's per-step env wrappers as a device pass
 * after the tick — BaseStatWrapper (reinforcement_learning/stat_wrapper.py:9-185) plus the
 * agent reward wrappers' reward shaping and ActionTargets edits. ---- */
#define NMMO_WRAP_BASE 0       /* BaseStatWrapper only (reward_terminated_truncated_info = id) */
#define NMMO_WRAP_START_KIT 1  /* agent_zoo/neurips23_start_kit/reward_wrapper.py */
#define NMMO_WRAP_TAKERU 2     /* agent_zoo/takeru/reward_wrapper.py */
#define NMMO_WRAP_YAOFENG 3    /* agent_zoo/yaofeng/reward_wrapper.py */
typedef struct NmmoWrapperConfig {
  int32_t kind;                       /* NMMO_WRAP_* */
  int32_t use_custom_reward;          /* stat_wrapper.py:17,77-86 */
  int32_t eval_mode;                  /* stat_wrapper.py:13,165-167: return = max progress */
  int32_t clip_unique_event;          /* start kit / takeru explore-bonus clip (3) */
  int32_t disable_give;               /* takeru / yaofeng: Give/GiveGold masks -> noop only */
  int32_t donot_attack_dangerous_npc; /* yaofeng: Attack.Target off for npc_type > 1 rows */
  double heal_bonus_weight, explore_bonus_weight;            /* start kit (+ takeru explore) */
  double hp_bonus_weight, exp_bonus_weight, defense_bonus_weight, attack_bonus_weight,
      gold_bonus_weight, custom_bonus_scale;                 /* yaofeng */
} NmmoWrapperConfig;

/* Per-agent episode record written on the step the agent is terminated or truncated (the
 * info dict of stat_wrapper.py:118-185). `performed` bit k = info["stats"]["event/<name>"] for
 * name in eat_food, drink_water, score_hit, player_kill, consume_item, harvest_item, list_item,
 * buy_item, equip_armor, equip_weapon, equip_tool, equip_ammo, harvest_weapon. */
typedef struct NmmoAgentInfo {
  int32_t done;                /* 1 on the agent's final step (term or trunc), else 0 */
  int32_t length;              /* info["length"] = realm.tick */
  double ret;                  /* info["return"] (eval_mode: the task's max progress) */
  double max_progress;         /* task._max_progress (info["curriculum"]) */
  int32_t reward_signal_count; /* task.reward_signal_count */
  int32_t task_completed;
  int32_t cod_attacked, cod_starved, cod_dehydrated;
  int32_t max_combat_level, max_harvest_skill_ammo, max_harvest_skill_consum;
  uint32_t performed;
  int32_t max_progress_to_center, earned_gold, max_damage;
  int32_t max_item_level[5];   /* armor, weapon, tool, ammo, consumable; -1 = key absent */
  int32_t agent_kill_count, npc_kill_count, unique_events;
} NmmoAgentInfo;

/* Per-agent wrapper state (nmmo_get_wrapper_state, parity tests). */
typedef struct NmmoWrapState {
  double cum_reward;           /* BaseStatWrapper.cum_rewards */
  int32_t prev_count, curr_count; /* _unique_events prev/curr */
  int32_t prev_price;          /* start kit _history.prev_price */
  int32_t hp, exp, gold, dmg_inflicted_prev; /* yaofeng _data */
  int32_t dmg_inflicted;       /* history.damage_inflicted */
  uint32_t performed;          /* event-log accumulators of the episode (NmmoAgentInfo) */
  int32_t max_dist, earned_gold, max_damage;
  int32_t max_item_level[5];
  int32_t agent_kills, npc_kills;
  int32_t reserved;
} NmmoWrapState;
/* unique (event, type, level) tuples an agent has experienced: a bitset of
 * 17 codes x 18 types x 16 levels */
#define NMMO_UNIQ_WORDS 153

typedef struct NmmoConfig {
  int32_t abi_version;        /* must be NMMO_ABI_VERSION */
  int32_t player_n;           /* PLAYER_N 128 (environment.py:35, config.yaml:76); <= 128 */
  int32_t npc_n;              /* NPC_N 256 (environment.py:43, config.yaml:77); <= 256 */
  int32_t horizon;            /* HORIZON 1024 (environment.py:35) */
  int32_t map_n;              /* MAP_N 256 (environment.py:36) */
  int32_t spawn_immunity;     /* COMBAT_SPAWN_IMMUNITY 20 (environment.py:48) */
  int32_t early_stop_agent_num; /* BaseStatWrapper early stop (stat_wrapper.py:68-69), 0 = off */
  uint32_t resilient_u32;     /* RESOURCE_RESILIENT_POPULATION as a u32 threshold (0.2 -> 0x33333333) */
  uint32_t systems;           /* NMMO_SYS_* bitmask (environment.py:14-25) */
  int32_t obs_layout;         /* NMMO_OBS_* */
  int32_t task_embed_dim;     /* TASK_EMBED_DIM 2048 (environment.py:44) */
  int32_t task_num_tick;      /* default task TickGE(num_tick) (manual_curriculum.py:56) */
  int32_t event_cap;          /* event-log ring rows per env (SPEC.md §11); 0 = no event log */
  int32_t reserved0;
  uint64_t map_seed;          /* map-bank generator seed */
  uint64_t env_index_base;    /* global index of env 0 of this handle (rank sharding) */
} NmmoConfig;

typedef struct NmmoLayout {
  int32_t obs_elems;          /* per-agent elements of the flat obs (23,987) */
  int32_t act_heads;          /* 12 */
  int32_t act_dims[NMMO_N_ACTION_HEADS];
  /* flat obs offsets (pufferlib sorted-key order) */
  int32_t off_mask_attack_style, off_mask_attack_target, off_mask_buy, off_mask_destroy,
      off_mask_give_item, off_mask_give_target, off_mask_givegold_price, off_mask_givegold_target,
      off_mask_move, off_mask_sell_item, off_mask_sell_price, off_mask_use;
  int32_t off_agent_id, off_current_tick, off_entity, off_inventory, off_market, off_task, off_tile;
  int32_t entity_rows, entity_cols, inventory_rows, item_cols, market_rows, tile_rows, tile_cols;
  /* state blob geometry */
  int32_t slots;              /* player_n + npc_n */
  int32_t nf, ne;
  size_t state_bytes_per_env; /* see nmmo_get_state */
} NmmoLayout;

typedef struct NmmoHandle NmmoHandle;

/* Fill cfg with the reference defaults (environment.py:31-49 + config.yaml env:). */
NMMO_API void nmmo_default_config(NmmoConfig* cfg);
NMMO_API int nmmo_layout(const NmmoConfig* cfg, NmmoLayout* out);

/* Allocate the SoA state for n_envs envs on `device` and generate the map bank.
 * task_embedding: host fp16[task_embed_dim] used as every agent's Task obs (may be NULL). */
NMMO_API int nmmo_create(const NmmoConfig* cfg, int32_t n_envs, uint64_t seed, int32_t device,
                const uint16_t* task_embedding, NmmoHandle** out);
NMMO_API void nmmo_destroy(NmmoHandle* h);

/* Reset every env (env_seeds: host uint64[n_envs] or NULL = derive from the create seed). */
NMMO_API int nmmo_reset(NmmoHandle* h, const uint64_t* env_seeds, void* obs, uint8_t* mask, void* stream);

/* Ends the current episode of every env whose dev_env_mask[e] != 0 (device u8 [n_envs]): the
 * env's next nmmo_step resets it instead of stepping (the auto-reset path, rewards/flags 0),
 * exactly as if its previous step had ended the episode; the ended episode's agents are not
 * reported as truncated. This is the per-env `env.reset()` the reference's async worker pool
 * issues independently for each env (pufferlib vectorization, clean_pufferl.py:106-114,175);
 * bench.py uses it to stagger episode phases across envs. Enqueued on `stream` (no device
 * synchronisation; graph-capturable). */
NMMO_API int nmmo_end_episodes(NmmoHandle* h, const uint8_t* dev_env_mask, void* stream);

/* One tick of every env. actions: device int32 [n_envs][player_n][12]. Envs whose previous
 * step ended the episode are reset instead (pufferlib auto-reset), with rewards/flags 0.
 * obs: device float32 [n_envs][player_n][obs_elems] (NMMO_OBS_FLAT), the native layout
 * [n_envs] x (player_n x NMMO_NATIVE_ROW_BYTES + NMMO_NATIVE_MARKET_BYTES) (NMMO_OBS_NATIVE),
 * a wire buffer of nmmo_wire_max_bytes (NMMO_OBS_WIRE: header + records, SPEC.md §8c; its
 * bytes equal nmmo_wire_pack of the native obs of the same state), or NULL (no obs gather).
 * rew f32, term/trunc/mask u8: device [n_envs][player_n]. */
NMMO_API int nmmo_step(NmmoHandle* h, const int32_t* actions, void* obs, float* rew, uint8_t* term,
              uint8_t* trunc, uint8_t* mask, void* stream);

/* One tick of the listed envs only: pool.send(actions) to the envs the last recv() returned
 * under pufferlib's async env pool (env_pool=True, envs_per_batch < num_envs; config.yaml:35-38,
 * clean_pufferl.py:106-114,293,357), where the other envs keep their state and their last
 * outputs. env_ids: device int32 [n_ids], distinct ids in [0, n_envs) (an id outside the range is
 * dropped and recorded in the fault word as NMMO_FAULT_ENV_LIST | position << 8; duplicates are
 * a precondition violation). Every other argument has nmmo_step's full [n_envs] shape: only the
 * listed envs' rows of actions are read and of obs / rew / term / trunc / mask written (the pool
 * keeps each env's outputs until its next recv). Auto-reset, the wrapper layer and the counters
 * behave as in nmmo_step for the listed envs. Flat and native obs only (NMMO_E_INVALID for a
 * wire obs buffer: its header packs every env). Enqueued on `stream`; graph-capturable. */
NMMO_API int nmmo_step_envs(NmmoHandle* h, const int32_t* env_ids, int32_t n_ids, const int32_t* actions, void* obs,
                            float* rew, uint8_t* term, uint8_t* trunc, uint8_t* mask, void* stream);

/* The observation gather alone, over the envs' current state (what nmmo_step's obs argument
 * writes after the tick): nmmo_step(obs = NULL) followed by nmmo_observe(obs) on the same stream
 * gives the same bytes as nmmo_step(obs). Replaces nmmo.Env._compute_observations, the second
 * half of nmmo.Env.step; lets a caller with several handles order their
 * HBM-bound gathers apart from their ticks (bench.py --batches). Graph-capturable. */
NMMO_API int nmmo_observe(NmmoHandle* h, void* obs, void* stream);

/* Incremental obs rows. Most of a flat row is zero runs: rows of agents out of the realm (dead,
 * or not yet spawned) are all-zero (pufferlib's pad_agent_data), and an agent's row holds ~5 of
 * its 100 Entity rows, a few of the 1,024 Market rows and Buy.MarketItem entries, and a Task
 * embedding that changes only with its task. nmmo_obs_bind makes `obs` the handle's own obs
 * buffer: for it the handle remembers, per agent row, what it last wrote there (row all-zero;
 * the Entity rows, Market rows and Buy entries past which the row is zero; the task whose
 * embedding it holds) and stores only what differs from that. The buffer's bytes after every
 * call are the same as when every row is written in full (tests/test_gpu_zero_rows.py checks
 * them against such a handle). Native rows skip only all-zero rows. Any other buffer passed to
 * nmmo_reset / nmmo_step / nmmo_step_envs / nmmo_observe gets every row written in full. A bound
 * buffer is the handle's until it is unbound (obs = NULL) or the handle destroyed: a caller that
 * writes into it calls nmmo_obs_invalidate first (the next gather then writes every row in
 * full); nmmo_obs_invalidate_envs forgets only the rows of the listed envs (device int32
 * [n_ids], ids in [0, n_envs); ids outside are ignored) -- what a pool that handed those envs'
 * rows to a consumer that may edit them in place calls before their next gather (the
 * reference's start-kit TileEncoder edits its Tile input in place, baseline_policy.py:96-97;
 * nmmo_amd.vecenv.GpuVecEnv with obs_readonly=False). Binding synchronises the device and
 * forgets the previous binding; nmmo_set_tasks forgets the Task sections itself.
 * NMMO_OBS_REZERO=1 in the environment at nmmo_create turns the tracking off (A/B).
 * nmmo_set_obs_counter: when set, every obs gather adds into dev_counter (device u64
 * [n_envs][2] on the handle's device, one pair per env so the adds do not contend): [e][0] +=
 * rows it wrote for env e (rows of agents in the realm + rows zeroed), [e][1] += bytes it stored
 * for env e (flat: the sections written; native: whole rows); NULL disables.
 * nmmo_obs_invalidate / nmmo_obs_invalidate_envs are enqueued on `stream` and capture-safe. */
NMMO_API int nmmo_obs_bind(NmmoHandle* h, const void* obs);
NMMO_API int nmmo_obs_invalidate(NmmoHandle* h, void* stream);
NMMO_API int nmmo_obs_invalidate_envs(NmmoHandle* h, const int32_t* env_ids, int32_t n_ids, void* stream);
/* nmmo_obs_invalidate_envs scoped to the sections a consumer writes (`sections`, a mask of
 * NMMO_OBS_SEC_*): with NMMO_OBS_SEC_TILE alone only the listed envs' rows' Tile sections are
 * forgotten -- the next gather rewrites every Tile entry of those rows (and re-zeroes the Tile of
 * rows out of the realm) and stays incremental everywhere else: what the start-kit policy's
 * in-place edit of Tile[:, :, :2] needs (baseline_policy.py:96-97). Any other mask, or a handle
 * whose rows do not track the Tile section (native layout, slot counts not a multiple of 8),
 * forgets the listed envs' whole rows. env_ids NULL = every env (n_ids ignored). Enqueued on
 * `stream`; capture-safe. */
#define NMMO_OBS_SEC_TILE 1u
#define NMMO_OBS_SEC_ALL 0xFFFFFFFFu
NMMO_API int nmmo_obs_invalidate_sections(NmmoHandle* h, const int32_t* env_ids, int32_t n_ids, uint32_t sections,
                                          void* stream);
NMMO_API int nmmo_set_obs_counter(NmmoHandle* h, uint64_t* dev_counter);

/* Task table and per-player assignment (SPEC.md §12; nmmo.Env.reset(make_task_fn) /
 * agent_task_map). tasks: host [n_tasks] (1..NMMO_MAX_TASKS); embeddings: host fp16
 * [n_tasks][task_embed_dim] used as each player's Task obs (NULL = keep the create-time
 * embedding for every task); assign: host int32 [n_envs][player_n] task indices (NULL = all 0).
 * Takes effect for progress from the next step; call before nmmo_reset for whole episodes.
 * Synchronous. Default after create: one task TickGE(task_num_tick). */
NMMO_API int nmmo_set_tasks(NmmoHandle* h, const NmmoTask* tasks, int32_t n_tasks,
                            const uint16_t* embeddings, const int32_t* assign);
/* Task sampling at reset (nmmo.Env's curriculum sampling by TaskSpec.sampling_weight,
 * environment.py:48-49 CURRICULUM_FILE_PATH, curriculum_generation/manual_curriculum.py):
 * weights: host double [n_tasks] (>= 0, finite, positive sum; n_tasks = the current table's),
 * or NULL to keep fixed assignments. While set, every env reset (nmmo_reset and the in-step
 * auto-reset) draws each player's task index independently with probability w_i / sum(w):
 * u = Philox draw (SPEC §2, purpose 8, index = player) compared against the thresholds
 * floor(2^32 * (w_0 + .. + w_i) / sum(w)) (SPEC §12). The drawn index is the player's
 * assignment (nmmo_get_state). nmmo_set_tasks clears the weights. Synchronous. */
NMMO_API int nmmo_set_task_weights(NmmoHandle* h, const double* weights, int32_t n_tasks);

/* Wrapper layer (SPEC.md §13; replaces the RewardWrapper(BaseStatWrapper) that env_creator
 * puts around every nmmo.Env, environment.py:58): wc = NULL turns it off. While on, every
 * nmmo_step / nmmo_reset runs it after the tick: rewards are shaped in place, the obs
 * ActionTargets edits are applied, and dev_info (device NmmoAgentInfo [n_envs][player_n],
 * caller-owned) receives each agent's episode record on its final step (done = 0 elsewhere).
 * Needs the event log (event_cap > 0). Resets every env's wrapper state; synchronous. */
NMMO_API int nmmo_set_wrapper(NmmoHandle* h, const NmmoWrapperConfig* wc, NmmoAgentInfo* dev_info);
/* host NmmoWrapState [n_envs][player_n] + u32 [n_envs][player_n][NMMO_UNIQ_WORDS]. Synchronous. */
NMMO_API int nmmo_get_wrapper_state(NmmoHandle* h, NmmoWrapState* host_state, uint32_t* host_uniq);
/* Event rows the wrapper never saw since nmmo_set_wrapper because a tick logged more than
 * event_cap rows and the ring overwrote them (summed over envs). Non-zero means the unique-event
 * counts and episode stats diverge from the reference's BaseStatWrapper: raise event_cap.
 * Synchronous. */
NMMO_API int nmmo_get_wrapper_dropped(NmmoHandle* h, int64_t* total);

/* Native -> flat obs (SPEC.md §8b): native device [n_envs] x (player_n rows + market) as
 * written by nmmo_step under NMMO_OBS_NATIVE, flat device float32 [n_envs][player_n][obs_elems]
 * (the pufferlib layout, bit-identical to what NMMO_OBS_FLAT writes). n_envs may be any count
 * of consecutive envs (e.g. a learner expanding gathered shards). Enqueued on `stream`. */
NMMO_API int nmmo_expand_obs(NmmoHandle* h, const void* native, float* flat, int32_t n_envs, void* stream);

/* Device buffer for the observation tensor: `bytes` of device memory mapped from 64-MB physical
 * chunks into one contiguous virtual range (hipMemCreate / hipMemMap). Large hipMalloc
 * allocations landed on physical placements whose write rate varied 5.4-6.5 TB/s under the obs
 * kernel's store pattern; chunk-mapped ones wrote at 6.5-6.6 TB/s every time. Synchronous;
 * NMMO_E_INVALID on a device without virtual memory management (the caller falls back to a
 * plain allocation). nmmo_dev_free synchronises the device first: call it at a sync point
 * (nmmo_amd/devmem.py defers it to one), never while a stream is capturing a graph. */
NMMO_API int nmmo_dev_alloc(int32_t device, uint64_t bytes, void** out);
NMMO_API int nmmo_dev_free(void* ptr);

/* ---- Wire encoding of native observations (SPEC.md §8c, v3) ----
 * For moving observations between GPUs (the learner gather of BASELINE config 5): the native
 * layout without its padding and repetition. A wire buffer of n_envs x player_n agents is
 *   header: int64 total bytes | int64 env payload offset [n_envs] | u16 agent count word
 *           [n_envs][player_n] (bit 15 in the realm, bits 0-6 visible entities, 7-10 items) |
 *           u16 market listings [n_envs] | u16 entity-table rows [n_envs], padded to 16 B
 *           (nmmo_wire_header_bytes);
 *   payload: per env, its entity table (the distinct Entity rows its records show, 31 int16
 *           each, ascending by the id's 16-bit pattern, padded to 16 B), one record per agent in
 *           the realm (slot order), then its listings (32 B each); a record (v4) is a 16-B head
 *           (int16 AgentId, CurrentTick, task index, tile row 0, tile col 0, m5, m6, gold), nv u16
 *           entity-table indices, ninv Inventory rows (16 int16), the 225 window materials at 4
 *           bits (114 B), the mask bit stream, zero pad to 16 B. The ActionTargets travel as what
 *           they are made of: m5 = nv | ninv << 7 | Exchange << 11 | (pp1 & 15) << 12, m6 = Style
 *           | Move (5 bits) << 1 | GoldPrice's count of leading ones << 6 | (pp1 >> 4) << 13 (pp1
 *           = 1 + the SellPrice entry the wrapper cleared, 0 = none), and the stream holds
 *           AttackTarget, GiveTarget, GoldTarget entries < nv then Destroy, GiveItem, SellItem,
 *           Use entries < ninv (3 nv + 4 ninv bits in whole u16 words; every later entry is 0,
 *           each noop 1).
 * The receiver reads `total` from the header; Buy.MarketItem is rebuilt from the listings. */
NMMO_API int64_t nmmo_wire_header_bytes(int32_t n_envs, int32_t player_n);
/* Upper bound of a wire buffer (every agent in the realm with 100 visible entities and 12 items,
 * full entity tables, every listing). */
NMMO_API int64_t nmmo_wire_max_bytes(int32_t n_envs, int32_t player_n);
/* Encodes `native` (the NMMO_OBS_NATIVE buffer of h's most recent obs gather; the per-agent
 * counts and the listing count come from that launch) into `wire` (device,
 * nmmo_wire_max_bytes). NMMO_E_INVALID when `native` is not the buffer the last obs gather
 * wrote, or a tick ran after it without an obs gather (the buffer no longer describes the
 * state the counts were taken from). Enqueued; the buffer's total size is its first int64
 * once the stream reaches it. */
NMMO_API int nmmo_wire_pack(NmmoHandle* h, const void* native, void* wire, void* stream);
/* Consistency check of a (received) wire buffer of n_envs x player_n agents: its announced
 * total against *dev_expect_total (device int64, or NULL to skip), the env payload offsets
 * against the count words, listing counts and entity tables, the count ranges, every record
 * head's AgentId / nv / ninv against its count word and its entity-table indices against the
 * table. ORs error bits into *dev_status (device int32: 1 total, 2 offsets, 4 count ranges,
 * 8 record heads, 16 entity-table indices; 0 = valid). Enqueued; needs no handle. */
NMMO_API int nmmo_wire_check(const void* wire, int32_t n_envs, int32_t player_n, const int64_t* dev_expect_total,
                             int32_t* dev_status, void* stream);
/* nmmo_wire_check over n_bufs (1..16) buffers in one launch (the learner root validating every
 * buffer a step received): wires / n_envs / dev_expect_totals are host arrays of n_bufs entries
 * (device buffers, their env counts, device int64 announced totals; dev_expect_totals NULL or an
 * entry NULL skips that comparison); the bits of all of them are OR-ed into *dev_status.
 * Enqueued; needs no handle. */
NMMO_API int nmmo_wire_check_many(const void* const* wires, const int32_t* n_envs,
                                  const int64_t* const* dev_expect_totals, int32_t n_bufs,
                                  int32_t player_n, int32_t* dev_status, void* stream);
/* The learner gather's sizes row of one step (nmmo_amd.distributed.WireExchange.post_sizes):
 * dev_row[j] = the announced total (first int64) of wires[j] for j < n_bufs (1..16 device wire
 * buffers), dev_row[n_bufs] = *dev_fault (a device int32 tick fault word, or 0 when NULL), and
 * *dev_fault is cleared. One launch, enqueued; graph-capturable; needs no handle. */
NMMO_API int nmmo_sizes_row(const void* const* wires, int32_t n_bufs, int32_t* dev_fault, int64_t* dev_row,
                            void* stream);
/* ---- the learner gather's point-to-point transfers (nmmo_amd.distributed.WireExchange) ----
 * One RCCL group of sends / receives per nmmo_p2p_group call, enqueued on `stream`, over a
 * communicator this library creates: nmmo_p2p_load resolves RCCL from the librccl the process
 * already has loaded (torch's: pass its path; loaded if it is not), rank 0 makes an id with
 * nmmo_p2p_unique_id (NMMO_P2P_ID_BYTES), every rank receives it (torch.distributed broadcast) and
 * calls nmmo_p2p_init with it -- collectively, like ncclCommInitRank. An op moves `bytes` bytes of
 * device memory at buf to (recv = 0) or from (recv = 1) rank `peer`. Replaces
 * torch.distributed.batch_isend_irecv on the gather's per-step path (~13.5 us of host time per op
 * there, ~1 us here). */
#define NMMO_P2P_ID_BYTES 128
typedef struct NmmoP2POp {
  void* buf;
  int64_t bytes;
  int32_t peer;
  int32_t recv;
} NmmoP2POp;
NMMO_API int nmmo_p2p_load(const char* librccl_path);
NMMO_API int nmmo_p2p_unique_id(void* id);
NMMO_API int nmmo_p2p_init(const void* id, int32_t world, int32_t rank, void** comm);
NMMO_API int nmmo_p2p_group(void* comm, const NmmoP2POp* ops, int32_t n_ops, void* stream);
NMMO_API int nmmo_p2p_destroy(void* comm);
/* The per-agent step records the learner gather ships beside each wire buffer: with dev_records
 * set (device, n_envs x player_n x 8 B; NULL = off), every nmmo_step that writes NMMO_OBS_WIRE obs
 * also writes, per agent, its reward (f32) | terminated | truncated | mask | 0 -- the step's rew /
 * term / trunc / mask outputs in one 8-B record, from the wire gather's own launch (instead of four
 * strided copies after it). dev_fault (device int32, or NULL): the same launch also does what
 * nmmo_fault_into(h, dev_fault) would after the step (a nonzero tick fault word is stored there
 * unless it already holds one). The pointers are read when each step is enqueued (a captured
 * step keeps the ones it saw). Replaces the caller-side packing of pufferlib's per-agent rewards /
 * dones / masks (clean_pufferl.py:305-318 consumes them per step). */
NMMO_API int nmmo_set_step_records(NmmoHandle* h, uint8_t* dev_records, int32_t* dev_fault);
/* Decodes a wire buffer of n_envs x player_n agents into the native layout (every byte of the
 * n_envs x (player_n x NMMO_NATIVE_ROW_BYTES + NMMO_NATIVE_MARKET_BYTES) buffer is written;
 * bit-identical to what the sender's nmmo_step wrote). Enqueued; needs no handle. */
NMMO_API int nmmo_wire_unpack(int32_t n_envs, int32_t player_n, const void* wire, void* native, void* stream);

/* Masked-uniform scripted actions from the current state (bench / tests). */
NMMO_API int nmmo_scripted_actions(NmmoHandle* h, uint64_t policy_seed, int32_t* actions, void* stream);

/* State blob: per env, [NMMO_NE int32 env fields][NF*slots int16 entity table]
 * [slots int16 free-row ring][MAP_TILES u8 material][player_n*12 x 2 u32 items]
 * [12*player_n int16 item-row ring][player_n int32 task index][player_n NmmoTaskState];
 * envs concatenated. Synchronous. */
NMMO_API int nmmo_get_state(NmmoHandle* h, void* host_buf, size_t nbytes);
NMMO_API int nmmo_set_state(NmmoHandle* h, const void* host_buf, size_t nbytes);
/* The generated map bank: host u8 [map_n][MAP_TILES]. Synchronous. */
NMMO_API int nmmo_get_map_bank(NmmoHandle* h, uint8_t* host_buf, size_t nbytes);
/* Replaces the map bank (maps loaded from PATH_MAPS/map{i}/map.npy, environment.py:33,41;
 * SURVEY.md §8f row 4): host u8 [map_n][MAP_TILES], every value a material id < 16. Envs pick
 * up their map at the next reset; the depleted-tile bitmap of the current state is re-derived
 * against the new bank. Synchronous. */
NMMO_API int nmmo_set_map_bank(NmmoHandle* h, const uint8_t* host_buf, size_t nbytes);

/* Kernel timing with HIP events recorded on the launch stream around each kernel of
 * nmmo_step (bench/profiling; off by default, up to 8192 steps buffered).
 * nmmo_read_timing synchronises, returns the summed milliseconds of the tick, obs and wrapper
 * kernels over the buffered steps in ms[0], ms[1], ms[2], their count in *n, and clears the
 * buffer. */
NMMO_API int nmmo_set_timing(NmmoHandle* h, int32_t enable);
/* Device-side rollout counters (the trainer's agent_SPS numerator, clean_pufferl.py:306):
 * when set, every nmmo_step / nmmo_reset adds into dev_counters (device u64 [3]):
 * [0] += sum of the mask it writes (agent-steps), [1] += envs whose episode ended,
 * [2] += event-log rows appended by stepped (not reset) envs.
 * NULL disables. The caller owns and zeroes the buffer; capture-safe. */
NMMO_API int nmmo_set_counters(NmmoHandle* h, uint64_t* dev_counters);
NMMO_API int nmmo_read_timing(NmmoHandle* h, double* ms /* [3] */, int32_t* n);
/* Tick fault word: every round loop of the tick (attack, Buy and Give rounds; SPEC §9 conflict
 * rounds) and the position-hash probe stop at a bound the serial-order argument never reaches
 * (rounds <= the number of pending actions). A launch that hits one records its first
 * (NMMO_FAULT_* | env << 8) here instead of hanging, and that env's tick is then not the serial
 * result. *fault = the word (0 = none); the word is cleared. Synchronous. */
#define NMMO_FAULT_ATTACK_ROUNDS 1
#define NMMO_FAULT_BUY_ROUNDS 2
#define NMMO_FAULT_GIVE_ROUNDS 3
#define NMMO_FAULT_HASH_PROBE 4
#define NMMO_FAULT_ENV_LIST 5   /* nmmo_step_envs: an env id outside [0, n_envs) (dropped) */
#define NMMO_FAULT_WIRE_SCAN 6  /* NMMO_OBS_WIRE: an env's payload offset never resolved (bounded wait) */
NMMO_API int nmmo_get_fault(NmmoHandle* h, int32_t* fault);
/* The fault word without a host sync: when the word is non-zero and *dev_dst (device int32) is
 * 0, the word is copied into it (the first fault of several handles is kept). The word is not
 * cleared. Enqueued on `stream`; graph-capturable (the learner gather ships it with its sizes). */
NMMO_API int nmmo_fault_into(NmmoHandle* h, int32_t* dev_dst, void* stream);
/* Test hook: sets the fault word to `fault` (synchronous), so a caller's fault checks can be
 * exercised without a faulting state. */
NMMO_API int nmmo_inject_fault(NmmoHandle* h, int32_t fault);

/* The event log of env `env` (realm.event_log.get_data): copies the most recent
 * min(retained, max_rows) rows, oldest first, into host_rows [max_rows][NMMO_EVENT_COLS] and
 * their count into *n_rows (retained = min(E_EVENT_COUNT, event_cap)). Synchronous. */
NMMO_API int nmmo_get_events(NmmoHandle* h, int32_t env, int32_t* host_rows, int32_t max_rows,
                             int32_t* n_rows);

/* ---- GPU-resident experience storage ----
 * The trainer-side buffers of the reference's clean_pufferl kept in HBM (the reference keeps
 * them as host numpy arrays and copies every step across PCIe):
 *   nmmo_exp_store   <- evaluate(): learner_mask / torch.where(...)[: batch_size - ptr + 1] and the
 *                       obs/values/actions/logprobs/rewards/dones stores + sort_keys
 *                                                  reinforcement_learning/clean_pufferl.py:331-346
 *                       (storage allocated at :182-197)
 *   nmmo_exp_sort    <- sorted(range(len(sort_keys)), key=sort_keys.__getitem__)  :414
 *   nmmo_exp_gae     <- the reversed advantage loop                              :424-436
 *   nmmo_gather_rows <- b_obs = obs_ary[b_idxs], b_actions/... and mb copies     :439-458
 * Every buffer is caller-owned device memory; rows are `capacity` = batch_size + 1 (:182). */
typedef struct NmmoExperience {
  int32_t capacity;     /* rows (batch_size + 1) */
  int32_t obs_elems;    /* flat obs row length (NmmoLayout.obs_elems) */
  int32_t n_slots;      /* env_id range: num_envs * player_n agent slots (:119) */
  float* obs;           /* [capacity][obs_elems] */
  int64_t* actions;     /* [capacity][12] (torch int64, :183) */
  float* logprobs;      /* [capacity] */
  float* rewards;       /* [capacity] */
  float* dones;         /* [capacity] */
  float* truncateds;    /* [capacity] (allocated by the reference, never written by evaluate) */
  float* values;        /* [capacity] */
  int32_t* env_id;      /* [capacity] sort key 1 */
  int32_t* step;        /* [capacity] sort key 2 (evaluate's step counter) */
  int32_t* seq;         /* [capacity] rank of the row among its env_id's rows */
  int32_t* slot_count;  /* [n_slots] rows stored per env_id; zero it with ptr to start a batch */
  int32_t* ptr;         /* [1] rows stored (clean_pufferl.py:200 ptr) */
  int32_t* status;      /* [1] or NULL: bit 0 set when a store met a selected row whose env_id is
                           outside [0, n_slots) (the row is dropped, nothing out of range is
                           written). Env ids must be distinct within one store (precondition).
                           Record storage: bit 1 a wire buffer without arena room or with an
                           implausible total, bit 3 one that failed the fused check, bit 4 one
                           inside the arena but not at its slot (each keeps no row). */
} NmmoExperience;

typedef struct NmmoStoreInput {
  int32_t n_rows;         /* agent rows of this recv (num_envs * player_n) */
  int32_t step;           /* evaluate's step counter; must increase between stores */
  const float* obs;       /* flat [n_rows][obs_elems], or NULL with native */
  const void* native;     /* NMMO_OBS_NATIVE buffer of n_rows / player_n envs (needs the handle) */
  const float* rewards;   /* [n_rows] */
  const uint8_t* dones;   /* [n_rows] (recv's d) */
  const uint8_t* mask;    /* [n_rows] learner mask (recv mask x policy-pool mask) */
  const int32_t* env_id;  /* [n_rows], distinct ids in [0, n_slots); NULL = env_id_base + row */
  int32_t env_id_base;
  const int32_t* actions; /* [n_rows][12] */
  const float* logprobs;  /* [n_rows] */
  const float* values;    /* [n_rows] */
  const void* wire;       /* NMMO_OBS_WIRE / nmmo_wire_pack buffer of n_rows / player_n envs (needs a
                             handle for the layout and task table), or NULL */
} NmmoStoreInput;

/* Compact experience observations (the learner side of the C5 gather): a stored
 * row's observation kept as the wire record it arrived in (SPEC.md §8c) instead of a 95,948-B
 * flat row. nmmo_exp_store_records copies the store's wire buffer (its `total` bytes) into a byte
 * arena behind a 16-B descriptor (int64 n_envs, int64 player_n) and records, per stored row, the
 * descriptor's arena offset and the row's agent index (env * player_n + agent) in that buffer;
 * nmmo_exp_gather_records expands rows to flat float32 rows when a minibatch needs them
 * (clean_pufferl.py:439-458), bit-identical to the rows nmmo_exp_store writes from the same wire
 * input. Every other experience field is stored as by nmmo_exp_store (x->obs may be NULL). */
typedef struct NmmoRecordStore {
  uint8_t* arena;        /* device bytes, 16-B aligned */
  int64_t arena_bytes;   /* its capacity */
  int64_t* arena_used;   /* device [1]: bytes used (zero it with the experience's ptr for a new batch) */
  int64_t* row_buf;      /* device [capacity]: arena offset of the row's buffer descriptor */
  int32_t* row_agent;    /* device [capacity]: env * player_n + agent in that buffer */
} NmmoRecordStore;

/* int32 scratch the storage calls need: max(n_rows + n_rows/512 + 8, n_slots).
 * nmmo_exp_scratch_ints_many: what nmmo_exp_store_records_many over n_inputs inputs of at most
 * max_rows rows each needs (its per-input block counts take more than the summed rows' count when
 * many small inputs meet few slots); NMMO_E_INVALID (< 0) for n_inputs outside 1..16. */
NMMO_API int64_t nmmo_exp_scratch_ints(int32_t max_rows, int32_t n_slots);
NMMO_API int64_t nmmo_exp_scratch_ints_many(int32_t n_inputs, int32_t max_rows, int32_t n_slots);
/* Appends the mask-selected rows of one recv (in row order, cut at the capacity) and advances
 * *ptr on the device; exactly one of obs / native / wire: native obs are expanded, and wire
 * records decoded, straight into the flat experience rows of the kept rows only (h = a handle
 * whose layout and task table produced them; NULL for flat obs). Enqueued on `stream`. */
NMMO_API int nmmo_exp_store(NmmoHandle* h, const NmmoExperience* x, const NmmoStoreInput* in,
                            int32_t* scratch, void* stream);
/* nmmo_exp_store for a wire input (in->wire, in->obs and in->native NULL) into compact record
 * storage: the mask-selected rows' fields as nmmo_exp_store, their observations as references
 * into rs's arena (which receives the buffer). When the arena has no room for the buffer, the
 * store keeps no row and ORs 2 into x->status. h: the wire handle (layout, task table).
 * Enqueued; scratch as nmmo_exp_store. */
NMMO_API int nmmo_exp_store_records(NmmoHandle* h, const NmmoExperience* x, const NmmoRecordStore* rs,
                                    const NmmoStoreInput* in, int32_t* scratch, void* stream);
/* nmmo_exp_store_records over n_inputs (1..16) wire inputs at once, stored in input order as
 * one store (the learner storing every rank's buffers of a step: a fixed number of launches
 * whatever the input count). field_stride > 0: each input's rewards / dones / mask are read
 * field_stride bytes apart per row (float at rewards, u8 at dones and mask; e.g. an 8-B packed
 * per-agent record), 0: packed arrays as in nmmo_exp_store. scratch: nmmo_exp_scratch_ints_many
 * ints. Enqueued. An input whose buffer already lies where it would be copied to (wire == arena +
 * the 16-B-aligned end of the arena's used part + 16 at its turn: received straight into the
 * arena) is stored in place, not copied; nmmo_exp_store_records likewise. */
NMMO_API int nmmo_exp_store_records_many(NmmoHandle* h, const NmmoExperience* x, const NmmoRecordStore* rs,
                                         const NmmoStoreInput* ins, int32_t n_inputs, int32_t field_stride,
                                         int32_t* scratch, void* stream);
/* nmmo_exp_store_records_many with the received-buffer check in front of its reservation pass (the
 * learner root of the C5 gather: one call validates every input as nmmo_wire_check_many does and
 * stores only the clean ones): each input's check bits (1 total vs *dev_expect_totals[i], 2 offsets, 4
 * count ranges, 8 record heads, 16 entity-table indices) are OR-ed into *dev_check_status (device
 * int32, or NULL), and an input with any bit set keeps no row (x->status bit 3). dev_expect_totals:
 * host array of n_inputs device int64 pointers (an entry or the array NULL skips that comparison).
 * check_mask: bit i set = check input i (an unchecked input, e.g. the root's own buffers, counts as
 * clean). dev_ctl: device int32 [NMMO_STORE_CTL_INTS], zero before the first call; every call leaves it
 * zero (one per stream: calls sharing it must not overlap). Any store of a buffer that lies inside
 * the arena but not at its reserved slot is refused (x->status bit 4), never copied. */
#define NMMO_STORE_CTL_INTS 16
NMMO_API int nmmo_exp_store_records_checked(NmmoHandle* h, const NmmoExperience* x, const NmmoRecordStore* rs,
                                            const NmmoStoreInput* ins, int32_t n_inputs, int32_t field_stride,
                                            const int64_t* const* dev_expect_totals, uint32_t check_mask,
                                            int32_t* dev_check_status, int32_t* dev_ctl, int32_t* scratch,
                                            void* stream);
/* out (device float32 [n][obs_elems]) = the flat rows of experience rows idx[0..n) (device
 * int32) stored by nmmo_exp_store_records; h: the handle whose task table the records' task
 * indices refer to. Enqueued. */
NMMO_API int nmmo_exp_gather_records(NmmoHandle* h, const NmmoExperience* x, const NmmoRecordStore* rs,
                                     const int32_t* idx, int32_t n, float* out, void* stream);
/* idxs (device int32 [*ptr]) = the row order sorted by (env_id, step). Enqueued. */
NMMO_API int nmmo_exp_sort(const NmmoExperience* x, int32_t* idxs, int32_t* scratch, void* stream);
/* advantages (device f32 [batch_size]) over idxs[0..batch_size], float32, the reference's op
 * order (bit-identical). Enqueued. */
NMMO_API int nmmo_exp_gae(const NmmoExperience* x, const int32_t* idxs, int32_t batch_size, double gamma,
                          double gae_lambda, float* advantages, void* stream);
/* out[k] = src[idx[k]] for n rows of row_bytes (a multiple of 4). Enqueued. */
NMMO_API int nmmo_gather_rows(const void* src, int64_t row_bytes, const int32_t* idx, int32_t n, void* out,
                              void* stream);

NMMO_API int32_t nmmo_n_envs(const NmmoHandle* h);
NMMO_API const char* nmmo_last_error(void);
NMMO_API int32_t nmmo_abi_version(void);
/* "src=<sha256 of the HIP sources + headers this library was compiled from> arch=gfx950 ...";
 * nmmo_amd/_native.py refuses a library whose source hash differs from the tree it ships in. */
NMMO_API const char* nmmo_build_info(void);

#ifdef __cplusplus
}
#endif
#endif /* NMMO_HIP_H */
