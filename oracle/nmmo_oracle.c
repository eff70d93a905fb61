/*
 * nmmo_oracle.c — TEST INFRASTRUCTURE ONLY. Serial CPU restatement of the Neural MMO tick
 * (SPEC.md v1), used as the parity checker for libnmmo_hip.so and as the `cpu_baseline`
 * ("port") leg of bench.py. The product path never links, loads or calls this file.
 *
 * PARITY vs REAL nmmo 2.1: UNPINNED. The simulator the reference calls (pip `nmmo>=2.1,<2.2`,
 * /root/reference/pyproject.toml:19) is not vendored and is absent from this image (SURVEY.md
 * §0, §8c); the reference's own tests hold no golden vectors for the step path.
 * This file restates nmmo 2.1's published algorithm as recalled (SPEC.md marks each decision)
 * and is pinned by (i) the layout facts the reference code hard-codes (tests/test_layout.py),
 * (ii) the heldout task embeddings decoded from the reference's .pkl fixtures
 * (tests/golden/), and (iii) golden rollouts committed under tests/golden/ (self-generated).
 *
 * Structure mirrors nmmo's Python (recalled module names in comments): Realm.step phases run in
 * entity insertion order, one entity at a time, exactly as the Python loops do. Reference call
 * sites of the path: env.step  reinforcement_learning/stat_wrapper.py:64, env.reset :51,
 * realm reads :122-185; obs consumers agent_zoo/neurips23_start_kit/baseline_policy.py:41-264.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/nmmo_hip.h"

/* ------------------------------------------------------------------ constants (SPEC §1) */
enum { BORDER = 16, CENTER = 128, SIZE = 160, LO = 16, HI = 143, VISION = 7, N_OBS = 100 };
enum { M_VOID, M_WATER, M_GRASS, M_SCRUB, M_FOILAGE, M_STONE, M_SLAG, M_ORE, M_STUMP, M_TREE,
       M_FRAGMENT, M_CRYSTAL, M_WEEDS, M_HERB, M_OCEAN, M_FISH };
enum { P_MAPSEL = 1, P_SPAWN_OFFSET = 2, P_RESILIENT = 3, P_NPC_SPAWN = 4, P_NPC_MOVE = 5,
       P_RESPAWN = 6 };
static const int EXP_THRESHOLD[10] = {0, 90, 250, 500, 900, 1500, 2400, 3700, 5500, 8000};
static const int DR[5] = {-1, 1, 0, 0, 0}, DC[5] = {0, 0, 1, -1, 0};

static int impassable(int m) {
  return m == M_VOID || m == M_WATER || m == M_STONE || m == M_OCEAN || m == M_FISH;
}
static uint32_t respawn_u32(int base) {
  switch (base) {
    case M_FOILAGE: return 107374182u;                 /* 0.025 */
    case M_TREE: case M_ORE: case M_CRYSTAL: return 429496729u; /* 0.1 */
    case M_HERB: case M_FISH: return 85899345u;        /* 0.02 */
    default: return 0u;
  }
}

/* ------------------------------------------------------------------ RNG (SPEC §2) */
static uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static void philox(const uint32_t ctr_in[4], uint32_t k0, uint32_t k1, uint32_t out[4]) {
  uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
  for (int r = 0; r < 10; r++) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c1 = (uint32_t)p1; c3 = (uint32_t)p0; c0 = n0; c2 = n2;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}
static void draw(uint64_t seed, uint32_t tick, uint32_t purpose, uint32_t index, uint32_t sub,
                 uint32_t out[4]) {
  uint32_t ctr[4] = {tick, purpose, index, sub};
  philox(ctr, (uint32_t)seed, (uint32_t)(seed >> 32), out);
}
static uint32_t U(uint32_t u, uint32_t n) { return (uint32_t)(((uint64_t)u * n) >> 32); }

/* ------------------------------------------------------------------ map bank (SPEC §3) */
static uint32_t h32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}
static uint64_t lattice(uint64_t seed, uint32_t m, uint32_t k, uint32_t gy, uint32_t gx) {
  uint32_t a = h32(m * 0x9E3779B1u + k * 0x85EBCA77u);
  uint32_t b = h32((uint32_t)(seed >> 32) ^ a ^ (gy * 0xC2B2AE3Du) ^ (gx * 0x27D4EB2Fu));
  return h32((uint32_t)seed ^ b) >> 16;
}
static uint64_t smooth(uint64_t t) { return (t * t * (196608u - 2 * t)) >> 32; }

static void generate_map(uint64_t seed, uint32_t m, uint8_t* out) {
  static const uint64_t amp[5] = {16, 8, 4, 2, 1};
  uint16_t* noise = (uint16_t*)malloc(NMMO_MAP_TILES * sizeof(uint16_t));
  int hist[256] = {0};
  for (int y = 0; y < SIZE; y++)
    for (int x = 0; x < SIZE; x++) {
      uint64_t acc = 0;
      for (uint32_t k = 0; k < 5; k++) {
        uint32_t S = 32u >> k, gy = y / S, gx = x / S;
        uint64_t sy = smooth(((uint64_t)(y % S) << 16) / S);
        uint64_t sx = smooth(((uint64_t)(x % S) << 16) / S);
        uint64_t v00 = lattice(seed, m, k, gy, gx), v01 = lattice(seed, m, k, gy, gx + 1);
        uint64_t v10 = lattice(seed, m, k, gy + 1, gx), v11 = lattice(seed, m, k, gy + 1, gx + 1);
        uint64_t a = (v00 * (65536 - sx) + v01 * sx) >> 16;
        uint64_t b = (v10 * (65536 - sx) + v11 * sx) >> 16;
        acc += amp[k] * ((a * (65536 - sy) + b * sy) >> 16);
      }
      noise[y * SIZE + x] = (uint16_t)(acc / 31);
      if (y >= LO && y <= HI && x >= LO && x <= HI) hist[noise[y * SIZE + x] >> 8]++;
    }
  /* per-map quantile thresholds: water 15 %, grass to 70 %, foilage to 85 %, stone above */
  int bw = 255, bg = 255, bf = 255, cum = 0;
  for (int b = 0; b < 256; b++) {
    cum += hist[b];
    if (bw == 255 && cum >= 2458) bw = b;
    if (bg == 255 && cum >= 11469) bg = b;
    if (bf == 255 && cum >= 13926) bf = b;
  }
  for (int t = 0; t < NMMO_MAP_TILES; t++) {
    int b = noise[t] >> 8;
    out[t] = b <= bw ? M_WATER : b <= bg ? M_GRASS : b <= bf ? M_FOILAGE : M_STONE;
  }
  free(noise);
  /* resource pass reads the noise-pass materials only */
  uint8_t* base = (uint8_t*)malloc(NMMO_MAP_TILES);
  memcpy(base, out, NMMO_MAP_TILES);
  for (int y = 1; y < SIZE - 1; y++)
    for (int x = 1; x < SIZE - 1; x++) {
      int t = y * SIZE + x;
      uint32_t r = h32((uint32_t)seed ^ h32(m * 0x9E3779B1u ^ 0xA5A5A5A5u ^ h32((uint32_t)t))) % 1000;
      if (base[t] == M_GRASS) {
        if (r < 20) out[t] = M_TREE;
        else if (r < 35) out[t] = M_ORE;
        else if (r < 45) out[t] = M_CRYSTAL;
        else if (r < 60) out[t] = M_HERB;
      } else if (base[t] == M_WATER && r < 150) {
        int land = !impassable(base[t - SIZE]) || !impassable(base[t + SIZE]) ||
                   !impassable(base[t - 1]) || !impassable(base[t + 1]);
        if (land) out[t] = M_FISH;
      }
    }
  free(base);
  for (int y = 0; y < SIZE; y++)
    for (int x = 0; x < SIZE; x++) {
      int t = y * SIZE + x;
      if (y < LO || y > HI || x < LO || x > HI) out[t] = M_VOID;
      else if (y == LO || y == HI || x == LO || x == HI) out[t] = M_GRASS;
    }
}

/* ------------------------------------------------------------------ flat obs layout */
/* pufferlib-0.7.3 flattening of nmmo's Dict obs: keys sorted at every level (SPEC §8). */
typedef struct {
  int mask_attack_style, mask_attack_target, mask_buy, mask_destroy, mask_give_item,
      mask_give_target, mask_givegold_price, mask_givegold_target, mask_move, mask_sell_item,
      mask_sell_price, mask_use, agent_id, current_tick, entity, inventory, market, task, tile,
      elems;
} FlatLayout;

static FlatLayout flat_layout(int task_dim) {
  FlatLayout L;
  int o = 0;
  L.mask_attack_style = o; o += 3;
  L.mask_attack_target = o; o += N_OBS + 1;
  L.mask_buy = o; o += 1024 + 1;
  L.mask_destroy = o; o += 12 + 1;
  L.mask_give_item = o; o += 12 + 1;
  L.mask_give_target = o; o += N_OBS + 1;
  L.mask_givegold_price = o; o += 99;
  L.mask_givegold_target = o; o += N_OBS + 1;
  L.mask_move = o; o += 5;
  L.mask_sell_item = o; o += 12 + 1;
  L.mask_sell_price = o; o += 99;
  L.mask_use = o; o += 12 + 1;
  L.agent_id = o; o += 1;
  L.current_tick = o; o += 1;
  L.entity = o; o += N_OBS * NMMO_N_ENTITY_COLS;
  L.inventory = o; o += 12 * 16;
  L.market = o; o += 1024 * 16;
  L.task = o; o += task_dim;
  L.tile = o; o += 225 * 3;
  L.elems = o;
  return L;
}

/* ------------------------------------------------------------------ oracle state */
typedef struct {
  NmmoConfig cfg;
  int n_envs, P, N, S; /* players, npc cap, slots */
  uint64_t seed;
  int32_t* env;        /* [n_envs][NE] */
  int16_t* ent;        /* [n_envs][NF][S] */
  int16_t* ring;       /* [n_envs][S] */
  uint8_t* mat;        /* [n_envs][TILES] */
  uint8_t* bank;       /* [map_n][TILES] */
  uint32_t* items;     /* [n_envs][P][INV][2] (SPEC §9 item words) */
  int16_t* iring;      /* [n_envs][INV*P] free item rows */
  int32_t* events;     /* [n_envs][event_cap][NMMO_EVENT_COLS] event-log rings (SPEC §11) */
  NmmoTask* tasks;     /* [n_tasks] task programs (SPEC §12) */
  int n_tasks, tev;    /* tev: some task term counts events */
  float* task_emb;     /* [n_tasks][task_embed_dim] Task obs per task */
  int32_t* assign;     /* [n_envs][P] task index of each player */
  NmmoTaskState* tstate; /* [n_envs][P] */
  uint64_t* task_cum;  /* [n_tasks] sampling thresholds (oracle_set_task_weights) or NULL */
} Oracle;

#define ENV(o, e) ((o)->env + (size_t)(e) * NMMO_NE)
#define ENT(o, e) ((o)->ent + (size_t)(e) * NMMO_NF * (o)->S)
#define FLD(t, f, s) (t)[(size_t)(f) * S + (s)]
#define INV NMMO_INV_SLOTS
#define INVP(o, e, p) ((o)->items + (((size_t)(e) * (o)->P + (p)) * INV) * 2)

static int sys_on(const Oracle* o, uint32_t s) { return (o->cfg.systems & s) != 0; }
static int level_at_exp(int exp) {
  int l = 0;
  for (int i = 0; i < 10; i++) l += exp >= EXP_THRESHOLD[i];
  return l;
}
static uint64_t env_seed(const int32_t* E) {
  return (uint64_t)(uint32_t)E[E_SEED_LO] | ((uint64_t)(uint32_t)E[E_SEED_HI] << 32);
}
static int linf(int r0, int c0, int r1, int c1) {
  int a = abs(r0 - r1), b = abs(c0 - c1);
  return a > b ? a : b;
}
static float half_to_float(uint16_t h) {
  uint32_t s = (uint32_t)(h >> 15) << 31, e = (h >> 10) & 31, m = h & 1023, bits;
  if (e == 0) {
    if (m == 0) bits = s;
    else { /* subnormal */
      int sh = 0;
      while (!(m & 1024)) { m <<= 1; sh++; }
      m &= 1023;
      bits = s | ((uint32_t)(127 - 15 - sh + 1) << 23) | (m << 13);
    }
  } else if (e == 31) bits = s | 0x7F800000u | (m << 13);
  else bits = s | ((e + 112) << 23) | (m << 13);
  float f;
  memcpy(&f, &bits, 4);
  return f;
}

/* ------------------------------------------------------------------ items (SPEC §9) */
enum { T_HAT = 2, T_TOP, T_BOTTOM, T_SPEAR, T_BOW, T_WAND, T_ROD, T_GLOVES, T_PICKAXE, T_AXE,
       T_CHISEL, T_WHETSTONE, T_ARROW, T_RUNES, T_RATION, T_POTION };
enum { P_BUY_ORDER = 7, P_TASK = 8 };
#define IT_TYPE(w) ((int)((w)[0] & 31))
#define IT_LEVEL(w) ((int)(((w)[0] >> 5) & 15))
#define IT_EQUIPPED(w) ((int)(((w)[0] >> 9) & 1))
#define IT_PRICE(w) ((int)(((w)[0] >> 10) & 127))
#define IT_LTICK(w) ((int)(((w)[0] >> 17) & 2047))
#define IT_QTY(w) ((int)((w)[1] & 0xFFFF))
#define IT_ROW(w) ((int)((w)[1] >> 16))

static int item_attack(int type, int level, int style) {
  if (type == T_SPEAR + style || type == T_WHETSTONE + style) return 5 + 5 * level;
  return 0;
}
static int item_defense(int type, int level) {
  if (type >= T_HAT && type <= T_BOTTOM) return 3 * level;
  if (type >= T_ROD && type <= T_CHISEL) return 2 * level;
  return 0;
}
static int equip_slot(int type) { /* hat top bottom held ammo; -1 consumable */
  if (type >= T_HAT && type <= T_BOTTOM) return type - T_HAT;
  if (type >= T_SPEAR && type <= T_CHISEL) return 3;
  if (type >= T_WHETSTONE && type <= T_RUNES) return 4;
  return -1;
}
static int inv_count(const uint32_t* inv) {
  int n = 0;
  while (n < INV && IT_TYPE(inv + 2 * n)) n++;
  return n;
}
static int inv_find(const uint32_t* inv, int row) {
  for (int k = 0; k < INV && IT_TYPE(inv + 2 * k); k++)
    if (IT_ROW(inv + 2 * k) == row) return k;
  return -1;
}
static void inv_remove(uint32_t* inv, int k) {
  for (int j = k; j < INV - 1; j++) { inv[2 * j] = inv[2 * j + 2]; inv[2 * j + 1] = inv[2 * j + 3]; }
  inv[2 * INV - 2] = inv[2 * INV - 1] = 0;
}
static void inv_insert_sorted(uint32_t* inv, uint32_t w0, uint32_t w1) { /* caller checked room */
  int n = inv_count(inv), k = n;
  while (k > 0 && IT_ROW(inv + 2 * (k - 1)) > (int)(w1 >> 16)) {
    inv[2 * k] = inv[2 * k - 2]; inv[2 * k + 1] = inv[2 * k - 1]; k--;
  }
  inv[2 * k] = w0; inv[2 * k + 1] = w1;
}
static int inv_stack_slot(const uint32_t* inv, int type, int level) {
  if (type < T_WHETSTONE || type > T_RUNES) return -1;
  for (int k = 0; k < INV && IT_TYPE(inv + 2 * k); k++)
    if (IT_TYPE(inv + 2 * k) == type && IT_LEVEL(inv + 2 * k) == level) return k;
  return -1;
}
static void free_item_row(Oracle* o, int e, int row) {
  int32_t* E = ENV(o, e);
  int16_t* ir = o->iring + (size_t)e * INV * o->P;
  ir[(E[E_ITEM_FREE_HEAD] + E[E_ITEM_FREE_COUNT]) % (INV * o->P)] = (int16_t)row;
  E[E_ITEM_FREE_COUNT]++;
}
static int alloc_item_row(Oracle* o, int e) {
  int32_t* E = ENV(o, e);
  int16_t* ir = o->iring + (size_t)e * INV * o->P;
  int row = ir[E[E_ITEM_FREE_HEAD]];
  E[E_ITEM_FREE_HEAD] = (E[E_ITEM_FREE_HEAD] + 1) % (INV * o->P);
  E[E_ITEM_FREE_COUNT]--;
  return row;
}
/* a brand-new item (harvest, NPC drop): stacks onto ammo, else a new row if there is room */
static void receive_new(Oracle* o, int e, int p, int type, int level) {
  uint32_t* inv = INVP(o, e, p);
  int k = inv_stack_slot(inv, type, level);
  if (k >= 0) { inv[2 * k + 1] += 1; return; }
  if (inv_count(inv) >= INV) return;
  int row = alloc_item_row(o, e);
  inv_insert_sorted(inv, (uint32_t)type | ((uint32_t)level << 5), 1u | ((uint32_t)row << 16));
}
/* an existing item moving into p's inventory (loot, give, buy), already unequipped/unlisted */
static void receive_moved(Oracle* o, int e, int p, uint32_t w0, uint32_t w1) {
  uint32_t* inv = INVP(o, e, p);
  uint32_t it[2] = {w0, w1};
  int k = inv_stack_slot(inv, IT_TYPE(it), IT_LEVEL(it));
  if (k >= 0) { inv[2 * k + 1] += (uint32_t)IT_QTY(it); free_item_row(o, e, IT_ROW(it)); return; }
  if (inv_count(inv) >= INV) { free_item_row(o, e, IT_ROW(it)); return; }
  inv_insert_sorted(inv, w0, w1);
}
static int has_room(Oracle* o, int e, int p, const uint32_t* it) {
  const uint32_t* inv = INVP(o, e, p);
  return inv_stack_slot(inv, IT_TYPE(it), IT_LEVEL(it)) >= 0 || inv_count(inv) < INV;
}
static void update_item_level(Oracle* o, int e, int p) {
  const int S = o->S;
  int16_t* T = ENT(o, e);
  const uint32_t* inv = INVP(o, e, p);
  int l = 0;
  for (int k = 0; k < INV && IT_TYPE(inv + 2 * k); k++)
    if (IT_EQUIPPED(inv + 2 * k)) l += IT_LEVEL(inv + 2 * k);
  FLD(T, F_ITEM_LEVEL, p) = (int16_t)l;
}
static int player_offense(Oracle* o, int e, int p, int style) {
  const uint32_t* inv = INVP(o, e, p);
  int a = 0;
  for (int k = 0; k < INV && IT_TYPE(inv + 2 * k); k++)
    if (IT_EQUIPPED(inv + 2 * k)) a += item_attack(IT_TYPE(inv + 2 * k), IT_LEVEL(inv + 2 * k), style);
  return a;
}
static int player_defense(Oracle* o, int e, int p) {
  const uint32_t* inv = INVP(o, e, p);
  int d = 0;
  for (int k = 0; k < INV && IT_TYPE(inv + 2 * k); k++)
    if (IT_EQUIPPED(inv + 2 * k)) d += item_defense(IT_TYPE(inv + 2 * k), IT_LEVEL(inv + 2 * k));
  return d;
}
/* level an item requires of its user (SPEC §9) */
static int requirement_level(const int16_t* T, int S, int p, int type) {
  if (type >= T_SPEAR && type <= T_WAND) return FLD(T, F_MELEE_LEVEL + 2 * (type - T_SPEAR), p);
  if (type >= T_WHETSTONE && type <= T_RUNES) return FLD(T, F_MELEE_LEVEL + 2 * (type - T_WHETSTONE), p);
  if (type >= T_ROD && type <= T_CHISEL) return FLD(T, F_FISHING_LEVEL + 2 * (type - T_ROD), p);
  if (type == T_RATION) return FLD(T, F_FISHING_LEVEL, p);
  if (type == T_POTION) return FLD(T, F_HERBALISM_LEVEL, p);
  int m = FLD(T, F_MELEE_LEVEL, p); /* armor: max combat level */
  if (FLD(T, F_RANGE_LEVEL, p) > m) m = FLD(T, F_RANGE_LEVEL, p);
  if (FLD(T, F_MAGE_LEVEL, p) > m) m = FLD(T, F_MAGE_LEVEL, p);
  return m;
}
static int usable(const int16_t* T, int S, int p, const uint32_t* it) {
  if (IT_PRICE(it)) return 0;
  if (equip_slot(IT_TYPE(it)) >= 0 && IT_EQUIPPED(it)) return 1;
  return IT_LEVEL(it) <= requirement_level(T, S, p, IT_TYPE(it));
}
/* returns the new level on a level-up, else 0 */
static int add_skill_exp(int16_t* T, int S, int p, int f_exp, int xp) {
  int ex = FLD(T, f_exp, p) + xp;
  FLD(T, f_exp, p) = (int16_t)ex;
  int nl = level_at_exp(ex);
  if (nl > FLD(T, f_exp - 1, p)) { FLD(T, f_exp - 1, p) = (int16_t)nl; return nl; }
  return 0;
}

/* ------------------------------------------------------------------ event log (SPEC §11) */
/* EventLogger.record: players only; row k of the episode at ring index (k-1) mod event_cap */
/* ------------------------------------------------------------------ tasks (SPEC §12) */
static int pred_counts_events(int pred) {
  return (pred >= PRED_COUNT_EVENT && pred <= PRED_DEFEAT_ENTITY) || pred == PRED_PRACTICE_EATING;
}

/* an event of player p feeds the event accumulators of p's task terms */
static void task_accumulate(Oracle* o, int e, int p, int code, int type, int level, int number,
                            int gold, int target) {
  const NmmoTask* t = &o->tasks[o->assign[(size_t)e * o->P + p]];
  NmmoTaskState* ts = &o->tstate[(size_t)e * o->P + p];
  for (int k = 0; k < 2; k++) {
    const NmmoTaskTerm* q = &t->term[k];
    int32_t* acc = ts->acc + 2 * k;
    switch (q->pred) {
      case PRED_COUNT_EVENT: if (code == q->a) acc[0] += 1; break;
      case PRED_PRACTICE_EATING: if (code == EV_EAT_FOOD) acc[0] += 1; break;
      case PRED_SCORE_HIT: if (code == EV_SCORE_HIT && type == q->a) acc[0] += 1; break;
      case PRED_HARVEST_ITEM: if (code == EV_HARVEST_ITEM && type == q->a && level >= q->b) acc[0] += number; break;
      case PRED_CONSUME_ITEM: if (code == EV_CONSUME_ITEM && type == q->a && level >= q->b) acc[0] += number; break;
      case PRED_LIST_ITEM: if (code == EV_LIST_ITEM && type == q->a && level >= q->b) acc[0] += number; break;
      case PRED_BUY_ITEM: if (code == EV_BUY_ITEM && type == q->a && level >= q->b) acc[0] += number; break;
      case PRED_EARN_GOLD: if (code == EV_EARN_GOLD) acc[0] += gold; break;
      case PRED_SPEND_GOLD: if (code == EV_BUY_ITEM) acc[0] += gold; break;
      case PRED_MAKE_PROFIT:
        if (code == EV_EARN_GOLD) acc[0] += gold;
        if (code == EV_BUY_ITEM) acc[1] += gold;
        break;
      case PRED_DEFEAT_ENTITY:
        if (code == EV_PLAYER_KILL && ((q->a == 0 && target < 0) || (q->a == 1 && target > 0)) && level >= q->b)
          acc[0] += 1;
        break;
      default: break;
    }
  }
}

static void log_event(Oracle* o, int e, int p, int code, int type, int level, int number, int gold,
                      int target) {
  const int cap = o->cfg.event_cap;
  if (p < 0 || p >= o->P) return;
  if (o->tev) task_accumulate(o, e, p, code, type, level, number, gold, target);
  if (cap <= 0) return;
  int32_t* E = ENV(o, e);
  const int32_t id = ++E[E_EVENT_COUNT];
  int32_t* r = o->events + ((size_t)e * cap + (size_t)((id - 1) % cap)) * NMMO_EVENT_COLS;
  r[0] = id; r[1] = p + 1; r[2] = E[E_TICK] + 1; r[3] = code; r[4] = type; r[5] = level;
  r[6] = number; r[7] = gold; r[8] = target;
}
/* loot events are appended after all attack events of the tick (SPEC §11 order (7)) */
static __thread int32_t g_pend[128 * 16][7];
static __thread int g_npend;
static void pend_event(int p, int code, int type, int level, int number, int gold, int target) {
  int32_t* r = g_pend[g_npend++];
  r[0] = p; r[1] = code; r[2] = type; r[3] = level; r[4] = number; r[5] = gold; r[6] = target;
}
static void flush_pending(Oracle* o, int e) {
  for (int i = 0; i < g_npend; i++)
    log_event(o, e, g_pend[i][0], g_pend[i][1], g_pend[i][2], g_pend[i][3], g_pend[i][4],
              g_pend[i][5], g_pend[i][6]);
  g_npend = 0;
}
static int max_combat_level(const int16_t* T, int S, int s) {
  int l = FLD(T, F_MELEE_LEVEL, s);
  if (FLD(T, F_RANGE_LEVEL, s) > l) l = FLD(T, F_RANGE_LEVEL, s);
  if (FLD(T, F_MAGE_LEVEL, s) > l) l = FLD(T, F_MAGE_LEVEL, s);
  return l;
}

/* ------------------------------------------------------------------ reset (SPEC §4) */
static void npc_spawn(Oracle* o, int e, uint32_t tick);

static void reset_env(Oracle* o, int e, uint64_t seed, int episode) {
  const int S = o->S, P = o->P;
  int32_t* E = ENV(o, e);
  int16_t* T = ENT(o, e);
  uint8_t* mat = o->mat + (size_t)e * NMMO_MAP_TILES;
  uint32_t u[4];
  memset(E, 0, NMMO_NE * sizeof(int32_t));
  memset(T, 0, (size_t)NMMO_NF * S * sizeof(int16_t));
  E[E_SEED_LO] = (int32_t)(uint32_t)seed;
  E[E_SEED_HI] = (int32_t)(uint32_t)(seed >> 32);
  E[E_EPISODE] = episode;
  E[E_ENV_INDEX] = (int32_t)(o->cfg.env_index_base + (uint64_t)e);
  draw(seed, 0, P_MAPSEL, 0, 0, u);
  E[E_MAP_ID] = (int32_t)U(u[0], (uint32_t)o->cfg.map_n);
  memcpy(mat, o->bank + (size_t)E[E_MAP_ID] * NMMO_MAP_TILES, NMMO_MAP_TILES);
  draw(seed, 0, P_SPAWN_OFFSET, 0, 0, u);
  uint32_t off = U(u[0], 508);
  for (int i = 0; i < P; i++) {
    uint32_t p = (off + (uint32_t)(i * 508 / P)) % 508, side = p / 127, k = p % 127;
    int r = side == 0 ? LO : side == 1 ? LO + (int)k : side == 2 ? HI : HI - (int)k;
    int c = side == 0 ? LO + (int)k : side == 1 ? HI : side == 2 ? HI - (int)k : LO;
    draw(seed, 0, P_RESILIENT, (uint32_t)i, 0, u);
    FLD(T, F_ID, i) = (int16_t)(i + 1);
    FLD(T, F_ROW, i) = (int16_t)r;
    FLD(T, F_COL, i) = (int16_t)c;
    FLD(T, F_HEALTH, i) = 100;
    FLD(T, F_FOOD, i) = 100;
    FLD(T, F_WATER, i) = 100;
    for (int sk = 0; sk < 8; sk++) FLD(T, F_MELEE_LEVEL + 2 * sk, i) = 1;
    FLD(T, F_ALIVE, i) = 1;
    FLD(T, F_DS_ROW, i) = (int16_t)(i + 1);
    FLD(T, F_RESILIENT, i) = u[0] < o->cfg.resilient_u32;
  }
  int16_t* ring = o->ring + (size_t)e * S;
  for (int k = 0; k < S; k++) ring[k] = 0;
  for (int k = 0; k < o->N; k++) ring[k] = (int16_t)(P + 1 + k);
  E[E_FREE_HEAD] = 0;
  E[E_FREE_COUNT] = o->N;
  E[E_NPC_NEXT_ID] = -1;
  E[E_PLAYERS_ALIVE] = P;
  memset(INVP(o, e, 0), 0, (size_t)P * INV * 8);
  int16_t* ir = o->iring + (size_t)e * INV * P;
  for (int k = 0; k < INV * P; k++) ir[k] = (int16_t)(k + 1);
  E[E_ITEM_FREE_HEAD] = 0;
  E[E_ITEM_FREE_COUNT] = INV * P;
  memset(&o->tstate[(size_t)e * P], 0, (size_t)P * sizeof(NmmoTaskState));
  if (o->task_cum) /* curriculum sampling (SPEC §12): each player draws its task independently */
    for (int i = 0; i < P; i++) {
      draw(seed, 0, P_TASK, (uint32_t)i, 0, u);
      int k = 0;
      while ((uint64_t)u[0] >= o->task_cum[k]) k++; /* task_cum[n_tasks - 1] = 2^32 */
      o->assign[(size_t)e * P + i] = k;
    }
  if (sys_on(o, NMMO_SYS_NPC)) npc_spawn(o, e, 0);
}

/* NPCManager.spawn (SPEC §5.7): up to 25 attempts, appended in spawn order. */
static void npc_spawn(Oracle* o, int e, uint32_t tick) {
  const int S = o->S, P = o->P;
  int32_t* E = ENV(o, e);
  int16_t* T = ENT(o, e);
  int16_t* ring = o->ring + (size_t)e * S;
  const uint8_t* mat = o->mat + (size_t)e * NMMO_MAP_TILES;
  uint64_t seed = env_seed(E);
  for (uint32_t a = 0; a < 25; a++) {
    if (E[E_NPC_COUNT] >= o->N) break;
    uint32_t u[4];
    draw(seed, tick, P_NPC_SPAWN, a, 0, u);
    int r = LO + (int)U(u[0], CENTER), c = LO + (int)U(u[1], CENTER);
    if (impassable(mat[r * SIZE + c])) continue;
    int dist = r - LO;
    if (HI - r < dist) dist = HI - r;
    if (c - LO < dist) dist = c - LO;
    if (HI - c < dist) dist = HI - c;
    int type = 20 * dist >= 1024 ? 3 : 20 * dist >= 640 ? 2 : 1;
    int style = (int)U(u[2], 3);
    int level = sys_on(o, NMMO_SYS_PROGRESSION) ? (9 * dist) / 64 + 1 : 0;
    int s = P + E[E_NPC_COUNT];
    for (int f = 0; f < NMMO_NF; f++) FLD(T, f, s) = 0;
    FLD(T, F_ID, s) = (int16_t)E[E_NPC_NEXT_ID];
    FLD(T, F_NPC_TYPE, s) = (int16_t)type;
    FLD(T, F_ROW, s) = (int16_t)r;
    FLD(T, F_COL, s) = (int16_t)c;
    FLD(T, F_HEALTH, s) = 100;
    FLD(T, F_FOOD, s) = 100;
    FLD(T, F_WATER, s) = 100;
    FLD(T, F_MELEE_LEVEL, s) = FLD(T, F_RANGE_LEVEL, s) = FLD(T, F_MAGE_LEVEL, s) = 1;
    if (level > 0) {
      FLD(T, F_MELEE_LEVEL + 2 * style, s) = (int16_t)level;
      FLD(T, F_MELEE_EXP + 2 * style, s) = (int16_t)EXP_THRESHOLD[level - 1];
    }
    if (sys_on(o, NMMO_SYS_EXCHANGE)) FLD(T, F_GOLD, s) = (int16_t)level;
    FLD(T, F_ALIVE, s) = 1;
    FLD(T, F_DS_ROW, s) = ring[E[E_FREE_HEAD]];
    FLD(T, F_STYLE, s) = (int16_t)style;
    FLD(T, F_NPC_LEVEL, s) = (int16_t)level;
    FLD(T, F_DROP_ARMOR, s) = (int16_t)U(u[3], 3);
    FLD(T, F_DROP_TOOL, s) = (int16_t)U(u[3] >> 2, 5);
    if (sys_on(o, NMMO_SYS_EQUIPMENT) && level > 0) { /* int(8 * (level - U[0,1))) */
      int eq = (int)((((uint64_t)level << 32) - u[3]) * 8 >> 32);
      FLD(T, F_EQUIP_OFFENSE, s) = FLD(T, F_EQUIP_DEFENSE, s) = (int16_t)eq;
    }
    E[E_FREE_HEAD] = (E[E_FREE_HEAD] + 1) % S;
    E[E_FREE_COUNT]--;
    E[E_NPC_NEXT_ID]--;
    E[E_NPC_COUNT]++;
  }
}

/* ------------------------------------------------------------------ visibility (SPEC §8) */
/* Entity.Query.window: entities in the realm within L∞ <= 7 in ascending datastore row order. */
static int visible_slots(const Oracle* o, int e, int p, int* out /* >= S */) {
  const int S = o->S;
  const int16_t* T = ENT(o, e);
  int r = FLD(T, F_ROW, p), c = FLD(T, F_COL, p), n = 0;
  /* slots ordered by datastore row: rows are unique among entities in the realm */
  int by_row[512];
  for (int k = 0; k <= S; k++) by_row[k] = -1;
  for (int s = 0; s < S; s++)
    if (FLD(T, F_ALIVE, s)) by_row[FLD(T, F_DS_ROW, s)] = s;
  for (int k = 1; k <= S; k++) {
    int s = by_row[k];
    if (s < 0) continue;
    if (linf(r, c, FLD(T, F_ROW, s), FLD(T, F_COL, s)) <= VISION) out[n++] = s;
  }
  return n;
}

/* ------------------------------------------------------------------ NPC AI (SPEC §6) */
static int player_slot_valid(const Oracle* o, const int16_t* T, int id, int r, int c) {
  const int S = o->S;
  if (id <= 0 || id > o->P) return 0;
  int s = id - 1;
  return FLD(T, F_ALIVE, s) && FLD(T, F_HEALTH, s) > 0 &&
         linf(r, c, FLD(T, F_ROW, s), FLD(T, F_COL, s)) <= VISION;
}

/* SPEC §6 v2 pathing: breadth-first search from the target tile (tr, tc) over the passable tiles
 * of the 15x15 window centred on the NPC at (r, c), 4-neighbour moves. Returns the first of
 * N, S, E, W whose neighbour of the NPC lies one step closer to the target, or -1 when the
 * target cannot be reached inside the window. */
static int window_bfs_step(const uint8_t* mat, int r, int c, int tr, int tc) {
  enum { W = 2 * VISION + 1 };
  int dist[W][W], qr[W * W], qc[W * W], head = 0, tail = 0;
  for (int i = 0; i < W; i++)
    for (int j = 0; j < W; j++) dist[i][j] = -1;
  const int si = tr - r + VISION, sj = tc - c + VISION;
  dist[si][sj] = 0;
  qr[tail] = si; qc[tail++] = sj;
  while (head < tail) {
    const int i = qr[head], j = qc[head++];
    for (int d = 0; d < 4; d++) {
      const int ni = i + DR[d], nj = j + DC[d];
      if (ni < 0 || ni >= W || nj < 0 || nj >= W || dist[ni][nj] >= 0) continue;
      if (impassable(mat[(r - VISION + ni) * SIZE + (c - VISION + nj)])) continue;
      dist[ni][nj] = dist[i][j] + 1;
      qr[tail] = ni; qc[tail++] = nj;
    }
  }
  const int here = dist[VISION][VISION];
  if (here < 0) return -1;
  for (int d = 0; d < 4; d++) {
    const int ni = VISION + DR[d], nj = VISION + DC[d];
    if (dist[ni][nj] == here - 1) return d;
  }
  return -1; /* unreachable: a neighbour one step closer always exists */
}

static void npc_decide(Oracle* o, int e, int n, int* move_dir, int* atk_target, int* atk_style) {
  const int S = o->S;
  int16_t* T = ENT(o, e);
  const uint8_t* mat = o->mat + (size_t)e * NMMO_MAP_TILES;
  const int32_t* E = ENV(o, e);
  int r = FLD(T, F_ROW, n), c = FLD(T, F_COL, n), id = FLD(T, F_ID, n);
  uint32_t u[4];
  draw(env_seed(E), (uint32_t)E[E_TICK], P_NPC_MOVE, (uint32_t)(-id), 0, u);
  *move_dir = -1;
  *atk_target = -1;
  *atk_style = FLD(T, F_STYLE, n);
  /* behavior.update */
  if (!player_slot_valid(o, T, FLD(T, F_ATTACKER_ID, n), r, c)) FLD(T, F_ATTACKER_ID, n) = 0;
  if (!player_slot_valid(o, T, FLD(T, F_TARGET_ID, n), r, c)) FLD(T, F_TARGET_ID, n) = 0;
  int type = FLD(T, F_NPC_TYPE, n), hunt = 0;
  if (type == 2 && FLD(T, F_ATTACKER_ID, n)) {
    FLD(T, F_TARGET_ID, n) = FLD(T, F_ATTACKER_ID, n);
    hunt = 1;
  } else if (type == 3) {
    if (!FLD(T, F_TARGET_ID, n)) { /* utils.closestTarget */
      int best = -1, bd = 1 << 30;
      for (int p = 0; p < o->P; p++) {
        if (!FLD(T, F_ALIVE, p) || FLD(T, F_HEALTH, p) <= 0) continue;
        int d = linf(r, c, FLD(T, F_ROW, p), FLD(T, F_COL, p));
        if (d <= VISION && d < bd) { bd = d; best = p; }
      }
      if (best >= 0) FLD(T, F_TARGET_ID, n) = FLD(T, F_ID, best);
    }
    hunt = FLD(T, F_TARGET_ID, n) != 0;
  }
  if (!hunt) { /* behavior.meander -> move.habitable */
    int cand[4], k = 0;
    for (int d = 0; d < 4; d++)
      if (!impassable(mat[(r + DR[d]) * SIZE + c + DC[d]])) cand[k++] = d;
    if (k) *move_dir = cand[U(u[0], (uint32_t)k)];
    return;
  }
  int ts = FLD(T, F_TARGET_ID, n) - 1;
  int tr = FLD(T, F_ROW, ts), tc = FLD(T, F_COL, ts);
  int dist = linf(r, c, tr, tc);
  if (dist == 0) {
    *move_dir = (int)U(u[1], 4);
  } else if (dist > 1 && (*move_dir = window_bfs_step(mat, r, c, tr, tc)) >= 0) {
    /* move.pathfind: first step of a shortest 4-neighbour path inside the NPC's 15x15 window
       (SPEC §6 v2, a bounded stand-in for nmmo's A*) */
  } else if (dist > 1) { /* target unreachable inside the window: greedy step (SPEC §6 v1 rule) */
    int dr = tr - r, dc = tc - c;
    int dir_r = dr > 0 ? 1 : 0, dir_c = dc > 0 ? 2 : 3;
    int first = abs(dr) >= abs(dc) ? dir_r : dir_c, second = abs(dr) >= abs(dc) ? dir_c : dir_r;
    int second_nz = abs(dr) >= abs(dc) ? dc != 0 : dr != 0;
    if (!impassable(mat[(r + DR[first]) * SIZE + c + DC[first]])) *move_dir = first;
    else if (second_nz && !impassable(mat[(r + DR[second]) * SIZE + c + DC[second]]))
      *move_dir = second;
  }
  if (dist <= 3) *atk_target = ts;
}

/* ------------------------------------------------------------------ combat (SPEC §1, §5.3) */
static int combat_level(const Oracle* o, const int16_t* T, int s) {
  const int S = o->S;
  int nsk = s < o->P ? 8 : 3, l = 0;
  for (int k = 0; k < nsk; k++)
    if (FLD(T, F_MELEE_LEVEL + 2 * k, s) > l) l = FLD(T, F_MELEE_LEVEL + 2 * k, s);
  return l;
}

/* a player killed its target: gold, then the victim's items (player) or its drops (NPC) */
static void loot(Oracle* o, int e, int x, int t) {
  const int S = o->S, P = o->P;
  int16_t* T = ENT(o, e);
  if (sys_on(o, NMMO_SYS_EXCHANGE)) {
    FLD(T, F_GOLD, x) = (int16_t)(FLD(T, F_GOLD, x) + FLD(T, F_GOLD, t));
    FLD(T, F_GOLD, t) = 0;
  }
  if (!sys_on(o, NMMO_SYS_ITEM)) return;
  if (t < P) {
    uint32_t* inv = INVP(o, e, t);
    while (IT_TYPE(inv)) {
      uint32_t w0 = inv[0] & 0x1FFu, w1 = inv[1]; /* unequipped, unlisted */
      w0 &= ~(1u << 9);
      pend_event(x, EV_LOOT_ITEM, IT_TYPE(inv), IT_LEVEL(inv), IT_QTY(inv), 0, FLD(T, F_ID, t));
      inv_remove(inv, 0);
      receive_moved(o, e, x, w0, w1);
    }
    update_item_level(o, e, t);
  } else {
    int lvl = FLD(T, F_NPC_LEVEL, t) > 0 ? FLD(T, F_NPC_LEVEL, t) : 1;
    if (sys_on(o, NMMO_SYS_EQUIPMENT)) {
      receive_new(o, e, x, T_HAT + FLD(T, F_DROP_ARMOR, t), lvl);
      pend_event(x, EV_LOOT_ITEM, T_HAT + FLD(T, F_DROP_ARMOR, t), lvl, 1, 0, FLD(T, F_ID, t));
    }
    if (sys_on(o, NMMO_SYS_PROFESSION)) {
      receive_new(o, e, x, T_ROD + FLD(T, F_DROP_TOOL, t), lvl);
      pend_event(x, EV_LOOT_ITEM, T_ROD + FLD(T, F_DROP_TOOL, t), lvl, 1, 0, FLD(T, F_ID, t));
    }
  }
}

static void attack_call(Oracle* o, int e, int x, int style, int t) {
  const int S = o->S, P = o->P;
  int16_t* T = ENT(o, e);
  const int32_t* E = ENV(o, e);
  if (!FLD(T, F_ALIVE, x) || FLD(T, F_HEALTH, x) <= 0) return;
  if (!FLD(T, F_ALIVE, t) || FLD(T, F_HEALTH, t) <= 0 || t == x) return;
  if (x < P && t < P && FLD(T, F_TIME_ALIVE, t) < o->cfg.spawn_immunity) return;
  if (x >= P && t >= P) return;
  if (linf(FLD(T, F_ROW, x), FLD(T, F_COL, x), FLD(T, F_ROW, t), FLD(T, F_COL, t)) > 3) return;
  FLD(T, F_ATTACKER_ID, t) = FLD(T, F_ID, x);
  int prog = sys_on(o, NMMO_SYS_PROGRESSION);
  int offense = prog ? 10 + 5 * FLD(T, F_MELEE_LEVEL + 2 * style, x) : 30;
  int defense = prog ? 5 * combat_level(o, T, t) : 0;
  if (sys_on(o, NMMO_SYS_EQUIPMENT)) {
    offense += x < P ? (sys_on(o, NMMO_SYS_ITEM) ? player_offense(o, e, x, style) : 0)
                     : FLD(T, F_EQUIP_OFFENSE, x);
    defense += t < P ? (sys_on(o, NMMO_SYS_ITEM) ? player_defense(o, e, t) : 0)
                     : FLD(T, F_EQUIP_DEFENSE, t);
  }
  /* combat.damage_multiplier: dominant = np.argmax of target exp; 1.0 when all equal */
  int e0 = FLD(T, F_MELEE_EXP, t), e1 = FLD(T, F_RANGE_EXP, t), e2 = FLD(T, F_MAGE_EXP, t);
  int mult4 = 4;
  int mx = e0 > e1 ? (e0 > e2 ? e0 : e2) : (e1 > e2 ? e1 : e2);
  int mn = e0 < e1 ? (e0 < e2 ? e0 : e2) : (e1 < e2 ? e1 : e2);
  if (mx != mn) {
    int dom = e0 == mx ? 0 : e1 == mx ? 1 : 2;
    static const int weakness[3] = {2, 0, 1}; /* melee<-mage, range<-melee, mage<-range */
    if (style == weakness[dom]) mult4 = 6;
  }
  int d4 = mult4 * offense - 4 * defense;
  if (d4 < offense) d4 = offense;
  int dmg = d4 >> 2, lvl_up = 0;
  if (x < P && prog) { /* Player.apply_damage -> skill.add_xp */
    int f = F_MELEE_EXP + 2 * style;
    FLD(T, f, x) = (int16_t)(FLD(T, f, x) + 6);
    int nl = level_at_exp(FLD(T, f, x));
    if (nl > FLD(T, f - 1, x)) { FLD(T, f - 1, x) = (int16_t)nl; lvl_up = nl; }
  }
  if (x < P && sys_on(o, NMMO_SYS_EQUIPMENT) && sys_on(o, NMMO_SYS_ITEM)) {
    uint32_t* inv = INVP(o, e, x); /* fire one unit of the equipped ammunition of this style */
    for (int k = 0; k < INV && IT_TYPE(inv + 2 * k); k++) {
      if (!IT_EQUIPPED(inv + 2 * k) || IT_TYPE(inv + 2 * k) != T_WHETSTONE + style) continue;
      inv[2 * k + 1] -= 1;
      if (IT_QTY(inv + 2 * k) == 0) {
        free_item_row(o, e, IT_ROW(inv + 2 * k));
        inv_remove(inv, k);
        update_item_level(o, e, x);
      }
      break;
    }
  }
  FLD(T, F_DAMAGE, t) = (int16_t)dmg;
  int h = FLD(T, F_HEALTH, t) - dmg;
  FLD(T, F_HEALTH, t) = (int16_t)(h < 0 ? 0 : h);
  log_event(o, e, x, EV_SCORE_HIT, style + 1, 0, dmg, 0, 0);
  if (lvl_up) log_event(o, e, x, EV_LEVEL_UP, style + 1, lvl_up, 0, 0, 0);
  if (FLD(T, F_HEALTH, t) == 0) {
    FLD(T, F_PLAYER_KILLS, x)++;
    log_event(o, e, x, EV_PLAYER_KILL, 0, max_combat_level(T, S, t), 0, 0, FLD(T, F_ID, t));
    if (x < P) loot(o, e, x, t);
  }
  FLD(T, F_LATEST_COMBAT_TICK, x) = FLD(T, F_LATEST_COMBAT_TICK, t) = (int16_t)(E[E_TICK] + 1);
}

static void move_call(Oracle* o, int e, int x, int d) {
  const int S = o->S;
  int16_t* T = ENT(o, e);
  const uint8_t* mat = o->mat + (size_t)e * NMMO_MAP_TILES;
  if (!FLD(T, F_ALIVE, x) || FLD(T, F_HEALTH, x) <= 0) return;
  int nr = FLD(T, F_ROW, x) + DR[d], nc = FLD(T, F_COL, x) + DC[d];
  if (impassable(mat[nr * SIZE + nc])) return;
  if (FLD(T, F_FREEZE, x) > 0) return;
  FLD(T, F_ROW, x) = (int16_t)nr;
  FLD(T, F_COL, x) = (int16_t)nc;
  int progress = 64 - linf(80, 80, nr, nc);
  if (progress > FLD(T, F_EXPLORATION, x)) {
    FLD(T, F_EXPLORATION, x) = (int16_t)progress;
    log_event(o, e, x, EV_GO_FARTHEST, 0, 0, progress, 0, 0);
  }
}

/* ------------------------------------------------------------------ observation (SPEC §8, §9) */
/* Item.Query.for_sale: every listed item, ascending item row (owner slot, inventory slot) */
static int market_list(Oracle* o, int e, int* own, int* slot) {
  int n = 0;
  for (int p = 0; p < o->P; p++) {
    const uint32_t* inv = INVP(o, e, p);
    for (int k = 0; k < INV && IT_TYPE(inv + 2 * k); k++) {
      if (!IT_PRICE(inv + 2 * k)) continue;
      int j = n++; /* insertion by row */
      while (j > 0 && IT_ROW(INVP(o, e, own[j - 1]) + 2 * slot[j - 1]) > IT_ROW(inv + 2 * k)) {
        own[j] = own[j - 1]; slot[j] = slot[j - 1]; j--;
      }
      own[j] = p; slot[j] = k;
    }
  }
  return n;
}

/* ActionTargets of player p as int8 in flat order (SPEC §8, §9) */
static void compute_masks(Oracle* o, int e, int p, const int* vis, int nv, const int* mown,
                          const int* mslot, int nm, int8_t* m /* [1586] */) {
  const FlatLayout L = flat_layout(0);
  const int S = o->S, P = o->P;
  const int16_t* T = ENT(o, e);
  const uint8_t* mat = o->mat + (size_t)e * NMMO_MAP_TILES;
  const uint32_t* inv = INVP(o, e, p);
  const int r = FLD(T, F_ROW, p), c = FLD(T, F_COL, p), gold = FLD(T, F_GOLD, p);
  const int item = sys_on(o, NMMO_SYS_ITEM), exch = sys_on(o, NMMO_SYS_EXCHANGE) && item;
  memset(m, 0, (size_t)L.agent_id);
  if (sys_on(o, NMMO_SYS_COMBAT))
    for (int k = 0; k < 3; k++) m[L.mask_attack_style + k] = 1;
  for (int i = 0; i < nv; i++) {
    int s = vis[i], d = linf(r, c, FLD(T, F_ROW, s), FLD(T, F_COL, s));
    if (sys_on(o, NMMO_SYS_COMBAT))
      m[L.mask_attack_target + i] = s != p && d <= 3 && !(s < P && FLD(T, F_TIME_ALIVE, s) < o->cfg.spawn_immunity);
    int same = s < P && s != p && d == 0;
    if (item) m[L.mask_give_target + i] = (int8_t)same;
    if (exch) m[L.mask_givegold_target + i] = (int8_t)same;
  }
  m[L.mask_attack_target + N_OBS] = 1;
  m[L.mask_give_target + N_OBS] = 1;
  m[L.mask_givegold_target + N_OBS] = 1;
  for (int d = 0; d < 5; d++)
    m[L.mask_move + d] = !impassable(mat[(r + DR[d]) * SIZE + c + DC[d]]);
  for (int k = 0; k < INV && IT_TYPE(inv + 2 * k); k++) {
    const uint32_t* it = inv + 2 * k;
    int free_ = !IT_EQUIPPED(it) && !IT_PRICE(it);
    if (item) {
      m[L.mask_use + k] = (int8_t)usable(T, S, p, it);
      m[L.mask_destroy + k] = (int8_t)free_;
      m[L.mask_give_item + k] = (int8_t)free_;
    }
    if (exch) m[L.mask_sell_item + k] = !IT_EQUIPPED(it);
  }
  m[L.mask_use + 12] = m[L.mask_destroy + 12] = m[L.mask_give_item + 12] = m[L.mask_sell_item + 12] = 1;
  if (exch) {
    for (int q = 0; q < 99; q++) {
      m[L.mask_givegold_price + q] = q < gold;
      m[L.mask_sell_price + q] = 1;
    }
    for (int j = 0; j < nm && j < 1024; j++) {
      const uint32_t* it = INVP(o, e, mown[j]) + 2 * mslot[j];
      m[L.mask_buy + j] = IT_PRICE(it) <= gold && mown[j] != p;
    }
  }
  m[L.mask_buy + 1024] = 1;
}

static void item_row16(const uint32_t* it, int owner_id, float* out) {
  int type = IT_TYPE(it), lvl = IT_LEVEL(it);
  out[0] = (float)IT_ROW(it);
  out[1] = (float)type;
  out[2] = (float)owner_id;
  out[3] = (float)lvl;
  out[4] = 0.f;
  out[5] = (float)IT_QTY(it);
  for (int st = 0; st < 3; st++) out[6 + st] = (float)item_attack(type, lvl, st);
  for (int st = 0; st < 3; st++) out[9 + st] = (float)item_defense(type, lvl);
  out[12] = type == T_POTION ? (float)(50 + 5 * lvl) : 0.f;
  out[13] = type == T_RATION ? (float)(50 + 5 * lvl) : 0.f;
  out[14] = (float)IT_EQUIPPED(it);
  out[15] = (float)IT_PRICE(it);
}

static void write_obs(Oracle* o, int e, float* obs_env /* [P][obs_elems] or NULL */) {
  if (!obs_env) return;
  const FlatLayout L = flat_layout(o->cfg.task_embed_dim);
  const int S = o->S, P = o->P;
  const int16_t* T = ENT(o, e);
  const int32_t* E = ENV(o, e);
  const uint8_t* mat = o->mat + (size_t)e * NMMO_MAP_TILES;
  int vis[512], mown[INV * 128], mslot[INV * 128];
  int8_t m[1586];
  int nm = market_list(o, e, mown, mslot);
  for (int p = 0; p < P; p++) {
    float* ob = obs_env + (size_t)p * L.elems;
    memset(ob, 0, sizeof(float) * (size_t)L.elems);
    if (!FLD(T, F_ALIVE, p)) continue;
    int r = FLD(T, F_ROW, p), c = FLD(T, F_COL, p);
    int nv = visible_slots(o, e, p, vis);
    if (nv > N_OBS) nv = N_OBS;
    compute_masks(o, e, p, vis, nv, mown, mslot, nm, m);
    for (int k = 0; k < L.agent_id; k++) ob[k] = (float)m[k];
    ob[L.agent_id] = (float)FLD(T, F_ID, p);
    ob[L.current_tick] = (float)E[E_TICK];
    for (int i = 0; i < nv; i++)
      for (int f = 0; f < NMMO_N_ENTITY_COLS; f++)
        ob[L.entity + i * NMMO_N_ENTITY_COLS + f] = (float)FLD(T, f, vis[i]);
    const uint32_t* inv = INVP(o, e, p);
    for (int k = 0; k < INV && IT_TYPE(inv + 2 * k); k++)
      item_row16(inv + 2 * k, FLD(T, F_ID, p), ob + L.inventory + 16 * k);
    for (int j = 0; j < nm && j < 1024; j++)
      item_row16(INVP(o, e, mown[j]) + 2 * mslot[j], FLD(T, F_ID, mown[j]), ob + L.market + 16 * j);
    const float* emb = o->task_emb + (size_t)o->assign[(size_t)e * P + p] * o->cfg.task_embed_dim;
    for (int k = 0; k < o->cfg.task_embed_dim; k++) ob[L.task + k] = emb[k];
    int w = 0;
    for (int dr = -VISION; dr <= VISION; dr++)
      for (int dc = -VISION; dc <= VISION; dc++, w++) {
        ob[L.tile + 3 * w + 0] = (float)(r + dr);
        ob[L.tile + 3 * w + 1] = (float)(c + dc);
        ob[L.tile + 3 * w + 2] = (float)mat[(r + dr) * SIZE + (c + dc)];
      }
  }
}

/* ------------------------------------------------------------------ task progress (SPEC §12) */
static double clip01(double x) { return x < 0.0 ? 0.0 : x > 1.0 ? 1.0 : x; }
static double per(int num, int den) { return (double)num / (double)(den > 0 ? den : 1); }

static double term_progress(Oracle* o, int e, int p, const NmmoTaskTerm* q, const int32_t* acc) {
  const int S = o->S;
  const int16_t* T = ENT(o, e);
  const int32_t* E = ENV(o, e);
  const uint32_t* inv = INVP(o, e, p);
  const int sk = q->a >= 1 && q->a <= 8 ? q->a - 1 : -1; /* skill id -> 0..7 */
  switch (q->pred) {
    case PRED_TICK_GE: return per(E[E_TICK], q->a);
    case PRED_PRACTICE_EATING: { /* curriculum_tutorial.py:45-57: num_eat * 0.06 (+0.1 at >= 1,
                                    +0.3 at >= 3), Python float arithmetic; norm() is the clip */
      double pr = (double)acc[0] * 0.06;
      if (acc[0] >= 1) pr += 0.1;
      if (acc[0] >= 3) pr += 0.3;
      return pr;
    }
    case PRED_COUNT_EVENT: case PRED_SCORE_HIT: return per(acc[0], q->b);
    case PRED_HARVEST_ITEM: case PRED_CONSUME_ITEM: case PRED_LIST_ITEM: case PRED_BUY_ITEM:
    case PRED_DEFEAT_ENTITY: return per(acc[0], q->c);
    case PRED_EARN_GOLD: case PRED_SPEND_GOLD: return per(acc[0], q->a);
    case PRED_MAKE_PROFIT: return per(acc[0] - acc[1], q->a);
    case PRED_HOARD_GOLD: return per(FLD(T, F_GOLD, p), q->a);
    case PRED_ATTAIN_SKILL: return sk >= 0 && FLD(T, F_MELEE_LEVEL + 2 * sk, p) >= q->b ? 1.0 : 0.0;
    case PRED_GAIN_EXPERIENCE: return sk >= 0 ? per(FLD(T, F_MELEE_EXP + 2 * sk, p), q->b) : 0.0;
    case PRED_EQUIP_ITEM:
      for (int k = 0; k < INV && IT_TYPE(inv + 2 * k); k++)
        if (IT_EQUIPPED(inv + 2 * k) && IT_TYPE(inv + 2 * k) == q->a && IT_LEVEL(inv + 2 * k) >= q->b) return 1.0;
      return 0.0;
    case PRED_OWN_ITEM: {
      int n = 0;
      for (int k = 0; k < INV && IT_TYPE(inv + 2 * k); k++)
        if (IT_TYPE(inv + 2 * k) == q->a && IT_LEVEL(inv + 2 * k) >= q->b) n += IT_QTY(inv + 2 * k);
      return per(n, q->c);
    }
    case PRED_INVENTORY_SPACE_GE: return INV - inv_count(inv) >= q->a ? 1.0 : 0.0;
    case PRED_OCCUPY_TILE: return FLD(T, F_ROW, p) == q->a && FLD(T, F_COL, p) == q->b ? 1.0 : 0.0;
    case PRED_CAN_SEE_TILE: {
      const uint8_t* mat = o->mat + (size_t)e * NMMO_MAP_TILES;
      const int r = FLD(T, F_ROW, p), c = FLD(T, F_COL, p);
      for (int dr = -VISION; dr <= VISION; dr++)
        for (int dc = -VISION; dc <= VISION; dc++)
          if (mat[(r + dr) * SIZE + c + dc] == q->a) return 1.0;
      return 0.0;
    }
    case PRED_CAN_SEE_AGENT: case PRED_CAN_SEE_GROUP: {
      /* SPEC §12: the target is in p's Entity obs after the tick (in the realm, L-inf <= 7,
         among the first 100 visible by datastore row); singleton teams in id order */
      const int P = o->P;
      const int id = q->a > 0 ? q->a : q->a == -1 ? (p == 0 ? P : p) : (p + 1 == P ? 1 : p + 2);
      const int t = id - 1;
      if (t < 0 || t >= P || !FLD(T, F_ALIVE, t)) return 0.0;
      const int r = FLD(T, F_ROW, p), c = FLD(T, F_COL, p);
      if (linf(r, c, FLD(T, F_ROW, t), FLD(T, F_COL, t)) > VISION) return 0.0;
      int before = 0;
      for (int s = 0; s < S; s++)
        if (FLD(T, F_ALIVE, s) && FLD(T, F_DS_ROW, s) < FLD(T, F_DS_ROW, t) &&
            linf(r, c, FLD(T, F_ROW, s), FLD(T, F_COL, s)) <= VISION)
          before++;
      return before < 100 ? 1.0 : 0.0;
    }
    case PRED_FULLY_ARMED: {
      if (q->a < 1 || q->a > 3) return 0.0;
      const int need[5] = {T_HAT, T_TOP, T_BOTTOM, T_SPEAR + q->a - 1, T_WHETSTONE + q->a - 1};
      for (int j = 0; j < 5; j++) {
        int ok = 0;
        for (int k = 0; k < INV && IT_TYPE(inv + 2 * k); k++)
          ok |= IT_EQUIPPED(inv + 2 * k) && IT_TYPE(inv + 2 * k) == need[j] && IT_LEVEL(inv + 2 * k) >= q->b;
        if (!ok) return 0.0;
      }
      return 1.0;
    }
    default: return 0.0;
  }
}

static double task_progress(Oracle* o, int e, int p) {
  const NmmoTask* t = &o->tasks[o->assign[(size_t)e * o->P + p]];
  const NmmoTaskState* ts = &o->tstate[(size_t)e * o->P + p];
  const double p0 = clip01(term_progress(o, e, p, &t->term[0], ts->acc));
  if (t->combine == NMMO_TASK_SINGLE) return p0;
  const double p1 = clip01(term_progress(o, e, p, &t->term[1], ts->acc + 2));
  const double v = t->combine == NMMO_TASK_SUM ? (double)t->term[0].weight * p0 + (double)t->term[1].weight * p1
                                               : p0 * p1;
  return clip01(v);
}

/* ------------------------------------------------------------------ step (SPEC §5) */
static void reset_outputs(Oracle* o, int e, float* rew, uint8_t* term, uint8_t* trunc,
                          uint8_t* mask) {
  for (int p = 0; p < o->P; p++) {
    size_t i = (size_t)e * o->P + p;
    if (rew) rew[i] = 0.f;
    if (term) term[i] = 0;
    if (trunc) trunc[i] = 0;
    if (mask) mask[i] = 1;
  }
}

static int acts(const int16_t* T, int S, int s) { return FLD(T, F_ALIVE, s) && FLD(T, F_HEALTH, s) > 0; }

/* the item row an InventoryItem index of the previous observation refers to (-1: none) */
static int decode_item(Oracle* o, int e, int p, int k) {
  const uint32_t* inv = INVP(o, e, p);
  return (k >= 0 && k < inv_count(inv)) ? IT_ROW(inv + 2 * k) : -1;
}

static void step_env(Oracle* o, int e, const int32_t* actions, float* obs, float* rew,
                     uint8_t* term, uint8_t* trunc, uint8_t* mask) {
  const int S = o->S, P = o->P;
  int32_t* E = ENV(o, e);
  int16_t* T = ENT(o, e);
  uint8_t* mat = o->mat + (size_t)e * NMMO_MAP_TILES;
  float* obs_env = obs ? obs + (size_t)e * P * flat_layout(o->cfg.task_embed_dim).elems : NULL;
  if (E[E_DONE]) { /* pufferlib auto-reset: this call resets instead of stepping */
    uint64_t ns = splitmix64(env_seed(E) ^ (0xD1B54A32D192ED03ull * (uint64_t)(E[E_EPISODE] + 1)));
    reset_env(o, e, ns, E[E_EPISODE] + 1);
    reset_outputs(o, e, rew, term, trunc, mask);
    write_obs(o, e, obs_env);
    return;
  }
  const uint32_t tick = (uint32_t)E[E_TICK];
  const int item = sys_on(o, NMMO_SYS_ITEM), exch = item && sys_on(o, NMMO_SYS_EXCHANGE);
  const int prof = item && sys_on(o, NMMO_SYS_PROFESSION);
  int present[128], move_dir[512], atk_t[512], atk_s[512], vis[512];
  int use_row[128], destroy_row[128], give_row[128], give_t[128], gg_t[128], gg_amt[128];
  int sell_row[128], sell_price[128], buy_row[128];
  int mown[INV * 128], mslot[INV * 128];
  for (int s = 0; s < S; s++) move_dir[s] = atk_t[s] = -1, atk_s[s] = 0;
  for (int p = 0; p < P; p++) {
    present[p] = FLD(T, F_ALIVE, p);
    use_row[p] = destroy_row[p] = give_row[p] = give_t[p] = gg_t[p] = sell_row[p] = buy_row[p] = -1;
    gg_amt[p] = sell_price[p] = 0;
  }
  const int nm = exch ? market_list(o, e, mown, mslot) : 0;

  /* 0. Env._validate_actions: deserialize against the previous observation's state */
  for (int p = 0; p < P; p++) {
    if (!present[p]) continue;
    const int32_t* a = actions + ((size_t)e * P + p) * NMMO_N_ACTION_HEADS;
    if (a[8] >= 0 && a[8] < 5) move_dir[p] = a[8];
    int nv = visible_slots(o, e, p, vis);
    if (nv > N_OBS) nv = N_OBS;
    if (sys_on(o, NMMO_SYS_COMBAT) && a[0] >= 0 && a[0] < 3 && a[1] >= 0 && a[1] < nv) {
      atk_t[p] = vis[a[1]];
      atk_s[p] = a[0];
    }
    if (!item) continue;
    use_row[p] = decode_item(o, e, p, a[11]);
    destroy_row[p] = decode_item(o, e, p, a[3]);
    if (a[5] >= 0 && a[5] < nv) {
      give_row[p] = decode_item(o, e, p, a[4]);
      give_t[p] = give_row[p] >= 0 ? vis[a[5]] : -1;
    }
    if (!exch) continue;
    if (a[7] >= 0 && a[7] < nv && a[6] >= 0 && a[6] < 99) { gg_t[p] = vis[a[7]]; gg_amt[p] = a[6] + 1; }
    if (a[10] >= 0 && a[10] < 99) { sell_row[p] = decode_item(o, e, p, a[9]); sell_price[p] = a[10] + 1; }
    if (a[2] >= 0 && a[2] < nm && a[2] < 1024) buy_row[p] = IT_ROW(INVP(o, e, mown[a[2]]) + 2 * mslot[a[2]]);
  }
  /* 1. npcs.actions */
  if (sys_on(o, NMMO_SYS_NPC))
    for (int n = P; n < P + E[E_NPC_COUNT]; n++)
      npc_decide(o, e, n, &move_dir[n], &atk_t[n], &atk_s[n]);
  /* 2. players.update / npcs.update */
  for (int s = 0; s < P + E[E_NPC_COUNT]; s++) {
    if (!FLD(T, F_ALIVE, s)) continue;
    if (FLD(T, F_DAMAGE, s) == 0) FLD(T, F_ATTACKER_ID, s) = 0;
    FLD(T, F_DAMAGE, s) = 0;
    FLD(T, F_TIME_ALIVE, s)++;
    if (s >= P) {
      int h = FLD(T, F_HEALTH, s) + 1;
      FLD(T, F_HEALTH, s) = (int16_t)(h > 100 ? 100 : h);
      continue;
    }
    int r = FLD(T, F_ROW, s), c = FLD(T, F_COL, s), tile = r * SIZE + c;
    if (sys_on(o, NMMO_SYS_RESOURCE)) {
      int org = FLD(T, F_HEALTH, s), h = org;
      if (FLD(T, F_FOOD, s) > 50 && FLD(T, F_WATER, s) > 50) h = h + 10 > 100 ? 100 : h + 10;
      int dmg = FLD(T, F_RESILIENT, s) ? 5 : 10;
      if (FLD(T, F_FOOD, s) == 0) h = h - dmg < 0 ? 0 : h - dmg;
      if (FLD(T, F_WATER, s) == 0) h = h - dmg < 0 ? 0 : h - dmg;
      FLD(T, F_HEALTH, s) = (int16_t)h;
      FLD(T, F_HEALTH_RESTORE, s) = (int16_t)(h - org);
      int fd = FLD(T, F_FOOD, s) - 5;
      FLD(T, F_FOOD, s) = (int16_t)(fd < 0 ? 0 : fd);
      if (mat[tile] == M_FOILAGE) { /* Food.update -> harvest (depletes) */
        FLD(T, F_FOOD, s) = 100;
        mat[tile] = M_SCRUB;
        log_event(o, e, s, EV_EAT_FOOD, 0, 0, 0, 0, 0);
      }
      int wt = FLD(T, F_WATER, s) - 5;
      FLD(T, F_WATER, s) = (int16_t)(wt < 0 ? 0 : wt);
      if (mat[tile - SIZE] == M_WATER || mat[tile + SIZE] == M_WATER ||
          mat[tile - 1] == M_WATER || mat[tile + 1] == M_WATER) {
        FLD(T, F_WATER, s) = 100;
        log_event(o, e, s, EV_DRINK_WATER, 0, 0, 0, 0, 0);
      }
    }
    if (prof) { /* fishing, herbalism, prospecting, carving, alchemy (SPEC §9) */
      const uint32_t* inv = INVP(o, e, s);
      int held = -1, held_lvl = 1;
      for (int k = 0; k < INV && IT_TYPE(inv + 2 * k); k++)
        if (IT_EQUIPPED(inv + 2 * k) && equip_slot(IT_TYPE(inv + 2 * k)) == 3) {
          held = IT_TYPE(inv + 2 * k);
          held_lvl = IT_LEVEL(inv + 2 * k);
        }
      int nb[4] = {tile - SIZE, tile + SIZE, tile - 1, tile + 1}, got = 0;
      for (int q = 0; q < 4; q++)
        if (mat[nb[q]] == M_FISH) { mat[nb[q]] = M_OCEAN; got = 1; }
      if (got) {
        int lvl = held == T_ROD ? held_lvl : 1;
        receive_new(o, e, s, T_RATION, lvl);
        log_event(o, e, s, EV_HARVEST_ITEM, T_RATION, lvl, 1, 0, 0);
        int nl = add_skill_exp(T, S, s, F_FISHING_EXP, 30 * lvl);
        if (nl) log_event(o, e, s, EV_LEVEL_UP, 4, nl, 0, 0, 0);
      }
      static const int from[4] = {M_HERB, M_ORE, M_TREE, M_CRYSTAL};
      static const int to[4] = {M_WEEDS, M_SLAG, M_STUMP, M_FRAGMENT};
      static const int out[4] = {T_POTION, T_WHETSTONE, T_ARROW, T_RUNES};
      static const int tool[4] = {T_GLOVES, T_PICKAXE, T_AXE, T_CHISEL};
      static const int fexp[4] = {F_HERBALISM_EXP, F_PROSPECTING_EXP, F_CARVING_EXP, F_ALCHEMY_EXP};
      for (int q = 0; q < 4; q++) {
        if (mat[tile] != from[q]) continue;
        mat[tile] = (uint8_t)to[q];
        int lvl = held == tool[q] ? held_lvl : 1;
        receive_new(o, e, s, out[q], lvl);
        log_event(o, e, s, EV_HARVEST_ITEM, out[q], lvl, 1, 0, 0);
        int nl = add_skill_exp(T, S, s, fexp[q], (q == 0 ? 30 : 15) * lvl);
        if (nl) log_event(o, e, s, EV_LEVEL_UP, 5 + q, nl, 0, 0, 0);
      }
    }
  }
  /* 3. actions by priority, slot order (Buy: shuffled) */
  for (int p = 0; p < P && item; p++) { /* Use (10) */
    if (use_row[p] < 0 || !acts(T, S, p)) continue;
    uint32_t* inv = INVP(o, e, p);
    int k = inv_find(inv, use_row[p]);
    if (k < 0 || IT_PRICE(inv + 2 * k)) continue;
    uint32_t* it = inv + 2 * k;
    int type = IT_TYPE(it), lvl = IT_LEVEL(it), slot = equip_slot(type);
    if (slot >= 0) {
      if (IT_EQUIPPED(it)) it[0] &= ~(1u << 9);
      else if (lvl <= requirement_level(T, S, p, type)) {
        for (int j = 0; j < INV && IT_TYPE(inv + 2 * j); j++)
          if (IT_EQUIPPED(inv + 2 * j) && equip_slot(IT_TYPE(inv + 2 * j)) == slot) inv[2 * j] &= ~(1u << 9);
        it[0] |= 1u << 9;
        log_event(o, e, p, EV_EQUIP_ITEM, type, lvl, IT_QTY(it), 0, 0);
      }
      update_item_level(o, e, p);
    } else if (lvl <= requirement_level(T, S, p, type)) {
      int rs = 50 + 5 * lvl;
      if (type == T_RATION) {
        FLD(T, F_FOOD, p) = (int16_t)(FLD(T, F_FOOD, p) + rs > 100 ? 100 : FLD(T, F_FOOD, p) + rs);
        FLD(T, F_WATER, p) = (int16_t)(FLD(T, F_WATER, p) + rs > 100 ? 100 : FLD(T, F_WATER, p) + rs);
      } else {
        FLD(T, F_HEALTH, p) = (int16_t)(FLD(T, F_HEALTH, p) + rs > 100 ? 100 : FLD(T, F_HEALTH, p) + rs);
      }
      it[1] -= 1;
      log_event(o, e, p, EV_CONSUME_ITEM, type, lvl, 1, 0, 0);
      if (IT_QTY(it) == 0) { free_item_row(o, e, IT_ROW(it)); inv_remove(inv, k); }
    }
  }
  if (exch) { /* Buy (20): players in shuffled order */
    int order[128], key[128], n = 0;
    for (int p = 0; p < P; p++) {
      if (buy_row[p] < 0) continue;
      uint32_t u[4];
      draw(env_seed(E), tick, P_BUY_ORDER, (uint32_t)(p + 1), 0, u);
      int j = n++;
      while (j > 0 && ((uint32_t)key[j - 1] > u[0] || ((uint32_t)key[j - 1] == u[0] && order[j - 1] > p))) {
        key[j] = key[j - 1]; order[j] = order[j - 1]; j--;
      }
      key[j] = (int)u[0]; order[j] = p;
    }
    for (int i = 0; i < n; i++) {
      int b = order[i];
      if (!acts(T, S, b)) continue;
      int owner = -1, k = -1;
      for (int q = 0; q < P && owner < 0; q++) {
        int kk = inv_find(INVP(o, e, q), buy_row[b]);
        if (kk >= 0) { owner = q; k = kk; }
      }
      if (owner < 0 || owner == b) continue;
      uint32_t* it = INVP(o, e, owner) + 2 * k;
      int price = IT_PRICE(it);
      if (!price || FLD(T, F_GOLD, b) < price || !has_room(o, e, b, it)) continue;
      FLD(T, F_GOLD, b) = (int16_t)(FLD(T, F_GOLD, b) - price);
      FLD(T, F_GOLD, owner) = (int16_t)(FLD(T, F_GOLD, owner) + price);
      uint32_t w0 = it[0] & 0x1FFu, w1 = it[1];
      log_event(o, e, b, EV_BUY_ITEM, IT_TYPE(it), IT_LEVEL(it), IT_QTY(it), price, 0);
      log_event(o, e, owner, EV_EARN_GOLD, 0, 0, 0, price, 0);
      inv_remove(INVP(o, e, owner), k);
      receive_moved(o, e, b, w0, w1);
    }
  }
  for (int p = 0; p < P && item; p++) { /* Give, GiveGold (30) */
    if (!acts(T, S, p)) continue;
    int t = give_t[p];
    if (give_row[p] >= 0 && t >= 0 && t < P && t != p && acts(T, S, t) &&
        FLD(T, F_ROW, t) == FLD(T, F_ROW, p) && FLD(T, F_COL, t) == FLD(T, F_COL, p)) {
      uint32_t* inv = INVP(o, e, p);
      int k = inv_find(inv, give_row[p]);
      if (k >= 0 && !IT_EQUIPPED(inv + 2 * k) && !IT_PRICE(inv + 2 * k) && has_room(o, e, t, inv + 2 * k)) {
        uint32_t w0 = inv[2 * k], w1 = inv[2 * k + 1];
        log_event(o, e, p, EV_GIVE_ITEM, IT_TYPE(inv + 2 * k), IT_LEVEL(inv + 2 * k), IT_QTY(inv + 2 * k), 0,
                  FLD(T, F_ID, t));
        inv_remove(inv, k);
        receive_moved(o, e, t, w0, w1);
      }
    }
    t = gg_t[p];
    if (exch && t >= 0 && t < P && t != p && acts(T, S, t) && gg_amt[p] <= FLD(T, F_GOLD, p) &&
        FLD(T, F_ROW, t) == FLD(T, F_ROW, p) && FLD(T, F_COL, t) == FLD(T, F_COL, p)) {
      FLD(T, F_GOLD, p) = (int16_t)(FLD(T, F_GOLD, p) - gg_amt[p]);
      FLD(T, F_GOLD, t) = (int16_t)(FLD(T, F_GOLD, t) + gg_amt[p]);
      log_event(o, e, p, EV_GIVE_GOLD, 0, 0, 0, gg_amt[p], FLD(T, F_ID, t));
    }
  }
  for (int p = 0; p < P && item; p++) { /* Destroy (40) */
    if (destroy_row[p] < 0 || !acts(T, S, p)) continue;
    uint32_t* inv = INVP(o, e, p);
    int k = inv_find(inv, destroy_row[p]);
    if (k < 0 || IT_EQUIPPED(inv + 2 * k) || IT_PRICE(inv + 2 * k)) continue;
    log_event(o, e, p, EV_DESTROY_ITEM, IT_TYPE(inv + 2 * k), IT_LEVEL(inv + 2 * k), IT_QTY(inv + 2 * k), 0, 0);
    free_item_row(o, e, IT_ROW(inv + 2 * k));
    inv_remove(inv, k);
  }
  g_npend = 0;
  for (int s = 0; s < P + E[E_NPC_COUNT]; s++) /* Attack (50) */
    if (atk_t[s] >= 0) attack_call(o, e, s, atk_s[s], atk_t[s]);
  flush_pending(o, e); /* loot events after all attack events */
  for (int s = 0; s < P + E[E_NPC_COUNT]; s++) /* Move (60) */
    if (move_dir[s] >= 0) move_call(o, e, s, move_dir[s]);
  for (int p = 0; p < P && exch; p++) { /* Sell (70) */
    if (sell_row[p] < 0 || !acts(T, S, p)) continue;
    uint32_t* inv = INVP(o, e, p);
    int k = inv_find(inv, sell_row[p]);
    if (k < 0 || IT_EQUIPPED(inv + 2 * k)) continue;
    inv[2 * k] = (inv[2 * k] & 0x3FFu) | ((uint32_t)sell_price[p] << 10) | (tick << 17);
    log_event(o, e, p, EV_LIST_ITEM, IT_TYPE(inv + 2 * k), IT_LEVEL(inv + 2 * k), IT_QTY(inv + 2 * k),
              sell_price[p], 0);
  }
  /* 4. cull (players then NPCs), rows appended to the free ring; compact NPC slots */
  int16_t* ring = o->ring + (size_t)e * S;
  int died[128] = {0};
  for (int s = 0; s < P + E[E_NPC_COUNT]; s++) {
    if (!FLD(T, F_ALIVE, s) || FLD(T, F_HEALTH, s) > 0) continue;
    ring[(E[E_FREE_HEAD] + E[E_FREE_COUNT]) % S] = FLD(T, F_DS_ROW, s);
    E[E_FREE_COUNT]++;
    FLD(T, F_ALIVE, s) = 0;
    if (s < P) {
      died[s] = 1;
      FLD(T, F_DIED_TICK, s) = (int16_t)(tick + 1);
      E[E_PLAYERS_ALIVE]--;
      log_event(o, e, s, EV_AGENT_CULLED, 0, 0, 0, 0, 0);
    }
  }
  for (int p = 0; p < P && item; p++) { /* unlooted items of the dead are destroyed */
    if (!died[p]) continue;
    uint32_t* inv = INVP(o, e, p);
    while (IT_TYPE(inv)) { free_item_row(o, e, IT_ROW(inv)); inv_remove(inv, 0); }
    FLD(T, F_ITEM_LEVEL, p) = 0;
  }
  int w = P;
  for (int s = P; s < P + E[E_NPC_COUNT]; s++) {
    if (!FLD(T, F_ALIVE, s)) continue;
    if (w != s)
      for (int f = 0; f < NMMO_NF; f++) FLD(T, f, w) = FLD(T, f, s);
    w++;
  }
  for (int s = w; s < P + E[E_NPC_COUNT]; s++)
    for (int f = 0; f < NMMO_NF; f++) FLD(T, f, s) = 0;
  E[E_NPC_COUNT] = w - P;
  /* 5. tick += 1 */
  E[E_TICK] = (int32_t)(tick + 1);
  /* 6. map.step: depleted tiles respawn */
  const uint8_t* base = o->bank + (size_t)E[E_MAP_ID] * NMMO_MAP_TILES;
  for (int t = 0; t < NMMO_MAP_TILES; t++) {
    if (mat[t] == base[t]) continue;
    uint32_t u[4];
    draw(env_seed(E), tick + 1, P_RESPAWN, (uint32_t)(t >> 2), 0, u);  /* one draw per 4 tiles */
    if (u[t & 3] < respawn_u32(base[t])) mat[t] = base[t];
  }
  /* exchange.step: listings older than 5 ticks expire */
  for (int p = 0; p < P && exch; p++) {
    uint32_t* inv = INVP(o, e, p);
    for (int k = 0; k < INV && IT_TYPE(inv + 2 * k); k++)
      if (IT_PRICE(inv + 2 * k) && (int)(tick + 1) - IT_LTICK(inv + 2 * k) > 5) inv[2 * k] &= 0x3FFu;
  }
  /* 7. NPC refill */
  if (sys_on(o, NMMO_SYS_NPC)) npc_spawn(o, e, tick + 1);
  /* 8. rewards, dones */
  int alive = E[E_PLAYERS_ALIVE];
  int done = alive == 0 || (int)(tick + 1) >= o->cfg.horizon || alive <= o->cfg.early_stop_agent_num;
  for (int p = 0; p < P; p++) {
    size_t i = (size_t)e * P + p;
    float rw = 0.f;
    if (present[p] && died[p]) {
      rw = -1.f;
    } else if (present[p]) { /* Task.compute_rewards: progress delta (SPEC §12) */
      NmmoTaskState* ts = &o->tstate[i];
      const double np = task_progress(o, e, p), d = np - ts->last;
      ts->last = np;
      if (np > ts->max_progress) ts->max_progress = np;
      if (d > 0.0) ts->signals++;
      if (np >= 1.0 && ts->completed_tick == 0) ts->completed_tick = E[E_TICK];
      rw = (float)d;
    }
    if (rew) rew[i] = rw;
    if (term) term[i] = (uint8_t)died[p];
    if (trunc) trunc[i] = (uint8_t)(done && FLD(T, F_ALIVE, p));
    if (mask) mask[i] = (uint8_t)present[p];
  }
  E[E_DONE] = done;
  write_obs(o, e, obs_env);
}

/* ------------------------------------------------------------------ scripted policy (SPEC §10) */
static void scripted_env(Oracle* o, int e, uint64_t pseed, int32_t* actions) {
  static const int seg_off[12] = {0, 3, 104, 1129, 1142, 1155, 1256, 1355, 1456, 1461, 1474, 1573};
  static const int seg_len[12] = {3, 101, 1025, 13, 13, 101, 99, 101, 5, 13, 99, 13};
  const int S = o->S, P = o->P;
  const int16_t* T = ENT(o, e);
  const int32_t* E = ENV(o, e);
  int vis[512], mown[INV * 128], mslot[INV * 128];
  int8_t m[1586];
  int nm = market_list(o, e, mown, mslot);
  for (int p = 0; p < P; p++) {
    int32_t* a = actions + ((size_t)e * P + p) * NMMO_N_ACTION_HEADS;
    for (int h = 0; h < NMMO_N_ACTION_HEADS; h++) a[h] = 0;
    if (!FLD(T, F_ALIVE, p)) continue;
    int nv = visible_slots(o, e, p, vis);
    if (nv > N_OBS) nv = N_OBS;
    compute_masks(o, e, p, vis, nv, mown, mslot, nm, m);
    uint32_t ctr[4] = {(uint32_t)E[E_TICK] + 2048u * (uint32_t)E[E_EPISODE],
                       (uint32_t)E[E_ENV_INDEX], (uint32_t)p, 0}, u[4];
    for (int h = 0; h < NMMO_N_ACTION_HEADS; h++) { /* uniform over the head's set mask bits */
      int n = 0;
      for (int k = 0; k < seg_len[h]; k++) n += m[seg_off[h] + k];
      if (n == 0) continue;
      ctr[3] = (uint32_t)h;
      philox(ctr, (uint32_t)pseed, (uint32_t)(pseed >> 32), u);
      int pick = (int)U(u[0], (uint32_t)n);
      for (int k = 0; k < seg_len[h]; k++)
        if (m[seg_off[h] + k] && pick-- == 0) { a[h] = k; break; }
    }
  }
}

/* ------------------------------------------------------------------ public oracle API */
#define EXPORT __attribute__((visibility("default")))

EXPORT int oracle_obs_elems(int task_dim) { return flat_layout(task_dim).elems; }
EXPORT int oracle_flat_offsets(int task_dim, int32_t* out /* [20] */) {
  FlatLayout L = flat_layout(task_dim);
  memcpy(out, &L, sizeof(L));
  return (int)(sizeof(L) / sizeof(int));
}
EXPORT size_t oracle_state_bytes_per_env(int slots, int players) {
  return NMMO_NE * 4 + (size_t)NMMO_NF * slots * 2 + (size_t)slots * 2 + NMMO_MAP_TILES +
         (size_t)players * INV * 8 + (size_t)INV * players * 2 + (size_t)players * 4 +
         (size_t)players * sizeof(NmmoTaskState);
}

EXPORT void* oracle_create(const NmmoConfig* cfg, int n_envs, uint64_t seed,
                           const uint16_t* task_emb) {
  if (!cfg || n_envs <= 0 || cfg->player_n <= 0 || cfg->player_n > 128 || cfg->npc_n < 0 ||
      cfg->npc_n > 256 || cfg->map_n <= 0 || cfg->task_embed_dim > 4096)
    return NULL;
  Oracle* o = (Oracle*)calloc(1, sizeof(Oracle));
  o->cfg = *cfg;
  o->n_envs = n_envs;
  o->P = cfg->player_n;
  o->N = (cfg->systems & NMMO_SYS_NPC) ? cfg->npc_n : 0;
  o->S = cfg->player_n + o->N; /* NPC slots exist only with the NPC system */
  o->seed = seed;
  o->env = (int32_t*)calloc((size_t)n_envs * NMMO_NE, 4);
  o->ent = (int16_t*)calloc((size_t)n_envs * NMMO_NF * o->S, 2);
  o->ring = (int16_t*)calloc((size_t)n_envs * o->S, 2);
  o->mat = (uint8_t*)calloc((size_t)n_envs * NMMO_MAP_TILES, 1);
  o->bank = (uint8_t*)malloc((size_t)cfg->map_n * NMMO_MAP_TILES);
  o->items = (uint32_t*)calloc((size_t)n_envs * o->P * INV * 2, 4);
  o->iring = (int16_t*)calloc((size_t)n_envs * INV * o->P, 2);
  o->events = (int32_t*)calloc((size_t)n_envs * (cfg->event_cap > 0 ? cfg->event_cap : 1) * NMMO_EVENT_COLS, 4);
  for (int m = 0; m < cfg->map_n; m++)
    generate_map(cfg->map_seed, (uint32_t)m, o->bank + (size_t)m * NMMO_MAP_TILES);
  o->n_tasks = 1; /* default: everyone runs TickGE(task_num_tick) */
  o->tasks = (NmmoTask*)calloc(1, sizeof(NmmoTask));
  o->tasks[0].term[0].pred = PRED_TICK_GE;
  o->tasks[0].term[0].a = cfg->task_num_tick;
  o->task_emb = (float*)calloc((size_t)(cfg->task_embed_dim > 0 ? cfg->task_embed_dim : 1), 4);
  for (int k = 0; k < cfg->task_embed_dim; k++) o->task_emb[k] = task_emb ? half_to_float(task_emb[k]) : 0.f;
  o->assign = (int32_t*)calloc((size_t)n_envs * o->P, 4);
  o->tstate = (NmmoTaskState*)calloc((size_t)n_envs * o->P, sizeof(NmmoTaskState));
  return o;
}

EXPORT void oracle_destroy(void* h) {
  Oracle* o = (Oracle*)h;
  if (!o) return;
  free(o->env); free(o->ent); free(o->ring); free(o->mat); free(o->bank);
  free(o->items); free(o->iring); free(o->events);
  free(o->tasks); free(o->task_emb); free(o->assign); free(o->tstate); free(o->task_cum); free(o);
}

EXPORT int oracle_reset(void* h, const uint64_t* env_seeds, float* obs, uint8_t* mask) {
  Oracle* o = (Oracle*)h;
  for (int e = 0; e < o->n_envs; e++) {
    uint64_t s = env_seeds ? env_seeds[e]
                           : splitmix64(o->seed ^ splitmix64(o->cfg.env_index_base + (uint64_t)e));
    reset_env(o, e, s, 0);
    reset_outputs(o, e, NULL, NULL, NULL, mask);
    write_obs(o, e, obs ? obs + (size_t)e * o->P * flat_layout(o->cfg.task_embed_dim).elems : NULL);
  }
  return 0;
}

/* as nmmo_end_episodes: the next step of each masked env resets it (auto-reset path) */
EXPORT int oracle_end_episodes(void* h, const uint8_t* env_mask) {
  Oracle* o = (Oracle*)h;
  for (int e = 0; e < o->n_envs; e++)
    if (env_mask[e]) ENV(o, e)[E_DONE] = 1;
  return 0;
}
/* one env's flat obs (P x obs_elems floats) from its current state, as the step/reset writes it */
EXPORT int oracle_write_obs(void* h, int env, float* obs_env) {
  Oracle* o = (Oracle*)h;
  if (env < 0 || env >= o->n_envs || !obs_env) return NMMO_E_INVALID;
  write_obs(o, env, obs_env);
  return 0;
}

/* Envs are independent; `env_lo..env_hi` lets the CPU baseline run one thread per env range. */
EXPORT int oracle_step_range(void* h, int env_lo, int env_hi, const int32_t* actions, float* obs,
                             float* rew, uint8_t* term, uint8_t* trunc, uint8_t* mask) {
  Oracle* o = (Oracle*)h;
  for (int e = env_lo; e < env_hi; e++) step_env(o, e, actions, obs, rew, term, trunc, mask);
  return 0;
}
EXPORT int oracle_step(void* h, const int32_t* actions, float* obs, float* rew, uint8_t* term,
                       uint8_t* trunc, uint8_t* mask) {
  Oracle* o = (Oracle*)h;
  return oracle_step_range(h, 0, o->n_envs, actions, obs, rew, term, trunc, mask);
}
EXPORT int oracle_scripted_actions_range(void* h, int env_lo, int env_hi, uint64_t pseed,
                                         int32_t* actions) {
  Oracle* o = (Oracle*)h;
  for (int e = env_lo; e < env_hi; e++) scripted_env(o, e, pseed, actions);
  return 0;
}
EXPORT int oracle_scripted_actions(void* h, uint64_t pseed, int32_t* actions) {
  Oracle* o = (Oracle*)h;
  return oracle_scripted_actions_range(h, 0, o->n_envs, pseed, actions);
}

EXPORT int oracle_get_state(void* h, void* buf, size_t nbytes) {
  Oracle* o = (Oracle*)h;
  size_t per = oracle_state_bytes_per_env(o->S, o->P);
  if (nbytes != per * (size_t)o->n_envs) return NMMO_E_SIZE;
  uint8_t* b = (uint8_t*)buf;
  for (int e = 0; e < o->n_envs; e++) {
    memcpy(b, ENV(o, e), NMMO_NE * 4); b += NMMO_NE * 4;
    memcpy(b, ENT(o, e), (size_t)NMMO_NF * o->S * 2); b += (size_t)NMMO_NF * o->S * 2;
    memcpy(b, o->ring + (size_t)e * o->S, (size_t)o->S * 2); b += (size_t)o->S * 2;
    memcpy(b, o->mat + (size_t)e * NMMO_MAP_TILES, NMMO_MAP_TILES); b += NMMO_MAP_TILES;
    memcpy(b, INVP(o, e, 0), (size_t)o->P * INV * 8); b += (size_t)o->P * INV * 8;
    memcpy(b, o->iring + (size_t)e * INV * o->P, (size_t)INV * o->P * 2); b += (size_t)INV * o->P * 2;
    memcpy(b, o->assign + (size_t)e * o->P, (size_t)o->P * 4); b += (size_t)o->P * 4;
    memcpy(b, o->tstate + (size_t)e * o->P, (size_t)o->P * sizeof(NmmoTaskState));
    b += (size_t)o->P * sizeof(NmmoTaskState);
  }
  return 0;
}
EXPORT int oracle_set_state(void* h, const void* buf, size_t nbytes) {
  Oracle* o = (Oracle*)h;
  size_t per = oracle_state_bytes_per_env(o->S, o->P);
  if (nbytes != per * (size_t)o->n_envs) return NMMO_E_SIZE;
  const uint8_t* b = (const uint8_t*)buf;
  for (int e = 0; e < o->n_envs; e++) {
    memcpy(ENV(o, e), b, NMMO_NE * 4); b += NMMO_NE * 4;
    memcpy(ENT(o, e), b, (size_t)NMMO_NF * o->S * 2); b += (size_t)NMMO_NF * o->S * 2;
    memcpy(o->ring + (size_t)e * o->S, b, (size_t)o->S * 2); b += (size_t)o->S * 2;
    memcpy(o->mat + (size_t)e * NMMO_MAP_TILES, b, NMMO_MAP_TILES); b += NMMO_MAP_TILES;
    memcpy(INVP(o, e, 0), b, (size_t)o->P * INV * 8); b += (size_t)o->P * INV * 8;
    memcpy(o->iring + (size_t)e * INV * o->P, b, (size_t)INV * o->P * 2); b += (size_t)INV * o->P * 2;
    memcpy(o->assign + (size_t)e * o->P, b, (size_t)o->P * 4); b += (size_t)o->P * 4;
    memcpy(o->tstate + (size_t)e * o->P, b, (size_t)o->P * sizeof(NmmoTaskState));
    b += (size_t)o->P * sizeof(NmmoTaskState);
  }
  return 0;
}
/* as nmmo_set_tasks (SPEC §12) */
EXPORT int oracle_set_tasks(void* h, const NmmoTask* tasks, int n_tasks, const uint16_t* emb,
                            const int32_t* assign) {
  Oracle* o = (Oracle*)h;
  if (!tasks || n_tasks < 1 || n_tasks > NMMO_MAX_TASKS) return NMMO_E_INVALID;
  for (int i = 0; i < n_tasks; i++)
    for (int k = 0; k < 2; k++)
      if (tasks[i].term[k].pred < 0 || tasks[i].term[k].pred >= NMMO_N_PREDICATES) return NMMO_E_INVALID;
  if (assign)
    for (size_t i = 0; i < (size_t)o->n_envs * o->P; i++)
      if (assign[i] < 0 || assign[i] >= n_tasks) return NMMO_E_INVALID;
  const int D = o->cfg.task_embed_dim;
  float* ne = (float*)calloc((size_t)n_tasks * (D > 0 ? D : 1), 4);
  for (int i = 0; i < n_tasks; i++)
    for (int k = 0; k < D; k++) ne[(size_t)i * D + k] = emb ? half_to_float(emb[(size_t)i * D + k]) : o->task_emb[k];
  free(o->task_emb);
  o->task_emb = ne;
  free(o->tasks);
  o->tasks = (NmmoTask*)malloc((size_t)n_tasks * sizeof(NmmoTask));
  memcpy(o->tasks, tasks, (size_t)n_tasks * sizeof(NmmoTask));
  o->n_tasks = n_tasks;
  free(o->task_cum); /* weights belong to the previous table */
  o->task_cum = NULL;
  o->tev = 0;
  for (int i = 0; i < n_tasks; i++)
    for (int k = 0; k < 2; k++) o->tev |= pred_counts_events(tasks[i].term[k].pred);
  for (size_t i = 0; i < (size_t)o->n_envs * o->P; i++) o->assign[i] = assign ? assign[i] : 0;
  return 0;
}

/* as nmmo_set_task_weights (SPEC §12): thresholds floor(2^32 * prefix / sum), last = 2^32 */
EXPORT int oracle_set_task_weights(void* h, const double* w, int n_tasks) {
  Oracle* o = (Oracle*)h;
  if (!w) { free(o->task_cum); o->task_cum = NULL; return 0; }
  if (n_tasks != o->n_tasks) return NMMO_E_SIZE;
  double sum = 0.0;
  for (int i = 0; i < n_tasks; i++) {
    if (!(w[i] >= 0.0) || w[i] > 1e300) return NMMO_E_INVALID;
    sum += w[i];
  }
  if (!(sum > 0.0)) return NMMO_E_INVALID;
  uint64_t* cum = (uint64_t*)malloc((size_t)n_tasks * 8);
  double acc = 0.0;
  for (int i = 0; i < n_tasks; i++) {
    acc += w[i];
    double f = floor(acc / sum * 4294967296.0);
    cum[i] = f >= 4294967296.0 ? (1ull << 32) : (uint64_t)f;
  }
  cum[n_tasks - 1] = 1ull << 32;
  free(o->task_cum);
  o->task_cum = cum;
  return 0;
}

/* the env's retained event rows, oldest first (as nmmo_get_events) */
EXPORT int oracle_get_events(void* h, int env, int32_t* rows, int max_rows, int* n_rows) {
  Oracle* o = (Oracle*)h;
  const int cap = o->cfg.event_cap;
  const int cnt = ENV(o, env)[E_EVENT_COUNT];
  int n = cap > 0 ? (cnt < cap ? cnt : cap) : 0;
  if (n > max_rows) n = max_rows;
  for (int i = 0; i < n; i++) {
    const int id = cnt - n + 1 + i;
    memcpy(rows + (size_t)i * NMMO_EVENT_COLS,
           o->events + ((size_t)env * cap + (size_t)((id - 1) % cap)) * NMMO_EVENT_COLS, NMMO_EVENT_COLS * 4);
  }
  *n_rows = n;
  return 0;
}

EXPORT int oracle_set_map_bank(void* h, const uint8_t* buf, size_t nbytes) {
  Oracle* o = (Oracle*)h;
  if (nbytes != (size_t)o->cfg.map_n * NMMO_MAP_TILES) return NMMO_E_SIZE;
  for (size_t i = 0; i < nbytes; i++)
    if (buf[i] >= 16) return NMMO_E_INVALID;
  memcpy(o->bank, buf, nbytes);
  return 0;
}

EXPORT int oracle_get_map_bank(void* h, uint8_t* buf, size_t nbytes) {
  Oracle* o = (Oracle*)h;
  if (nbytes != (size_t)o->cfg.map_n * NMMO_MAP_TILES) return NMMO_E_SIZE;
  memcpy(buf, o->bank, nbytes);
  return 0;
}
