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
  float task[4096];
} Oracle;

#define ENV(o, e) ((o)->env + (size_t)(e) * NMMO_NE)
#define ENT(o, e) ((o)->ent + (size_t)(e) * NMMO_NF * (o)->S)
#define FLD(t, f, s) (t)[(size_t)(f) * S + (s)]

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
  } else if (dist > 1) { /* move.pathfind: greedy step (SPEC §6 decision) */
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
    offense += FLD(T, F_EQUIP_OFFENSE, x);
    defense += FLD(T, F_EQUIP_DEFENSE, t);
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
  int dmg = d4 >> 2;
  if (x < P && prog) { /* Player.apply_damage -> skill.add_xp */
    int f = F_MELEE_EXP + 2 * style;
    FLD(T, f, x) = (int16_t)(FLD(T, f, x) + 6);
    int nl = level_at_exp(FLD(T, f, x));
    if (nl > FLD(T, f - 1, x)) FLD(T, f - 1, x) = (int16_t)nl;
  }
  FLD(T, F_DAMAGE, t) = (int16_t)dmg;
  int h = FLD(T, F_HEALTH, t) - dmg;
  FLD(T, F_HEALTH, t) = (int16_t)(h < 0 ? 0 : h);
  if (FLD(T, F_HEALTH, t) == 0) FLD(T, F_PLAYER_KILLS, x)++;
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
  if (progress > FLD(T, F_EXPLORATION, x)) FLD(T, F_EXPLORATION, x) = (int16_t)progress;
}

/* ------------------------------------------------------------------ observation (SPEC §8) */
static void write_obs(Oracle* o, int e, float* obs_env /* [P][obs_elems] or NULL */) {
  if (!obs_env) return;
  const FlatLayout L = flat_layout(o->cfg.task_embed_dim);
  const int S = o->S, P = o->P;
  const int16_t* T = ENT(o, e);
  const int32_t* E = ENV(o, e);
  const uint8_t* mat = o->mat + (size_t)e * NMMO_MAP_TILES;
  int vis[512];
  for (int p = 0; p < P; p++) {
    float* ob = obs_env + (size_t)p * L.elems;
    memset(ob, 0, sizeof(float) * (size_t)L.elems);
    if (!FLD(T, F_ALIVE, p)) continue;
    int r = FLD(T, F_ROW, p), c = FLD(T, F_COL, p);
    int nv = visible_slots(o, e, p, vis);
    if (nv > N_OBS) nv = N_OBS;
    /* ActionTargets */
    if (sys_on(o, NMMO_SYS_COMBAT))
      for (int k = 0; k < 3; k++) ob[L.mask_attack_style + k] = 1.f;
    for (int i = 0; i < nv && sys_on(o, NMMO_SYS_COMBAT); i++) {
      int s = vis[i];
      int ok = s != p && linf(r, c, FLD(T, F_ROW, s), FLD(T, F_COL, s)) <= 3 &&
               !(s < P && FLD(T, F_TIME_ALIVE, s) < o->cfg.spawn_immunity);
      ob[L.mask_attack_target + i] = ok ? 1.f : 0.f;
    }
    ob[L.mask_attack_target + N_OBS] = 1.f;
    ob[L.mask_buy + 1024] = 1.f;
    ob[L.mask_destroy + 12] = 1.f;
    ob[L.mask_give_item + 12] = 1.f;
    ob[L.mask_give_target + N_OBS] = 1.f;
    ob[L.mask_givegold_target + N_OBS] = 1.f;
    for (int d = 0; d < 5; d++)
      ob[L.mask_move + d] = impassable(mat[(r + DR[d]) * SIZE + c + DC[d]]) ? 0.f : 1.f;
    ob[L.mask_sell_item + 12] = 1.f;
    ob[L.mask_use + 12] = 1.f;
    ob[L.agent_id] = (float)FLD(T, F_ID, p);
    ob[L.current_tick] = (float)E[E_TICK];
    for (int i = 0; i < nv; i++)
      for (int f = 0; f < NMMO_N_ENTITY_COLS; f++)
        ob[L.entity + i * NMMO_N_ENTITY_COLS + f] = (float)FLD(T, f, vis[i]);
    for (int k = 0; k < o->cfg.task_embed_dim; k++) ob[L.task + k] = o->task[k];
    int w = 0;
    for (int dr = -VISION; dr <= VISION; dr++)
      for (int dc = -VISION; dc <= VISION; dc++, w++) {
        ob[L.tile + 3 * w + 0] = (float)(r + dr);
        ob[L.tile + 3 * w + 1] = (float)(c + dc);
        ob[L.tile + 3 * w + 2] = (float)mat[(r + dr) * SIZE + (c + dc)];
      }
  }
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
  int present[128], move_dir[512], atk_t[512], atk_s[512], vis[512];
  for (int s = 0; s < S; s++) move_dir[s] = atk_t[s] = -1, atk_s[s] = 0;
  for (int p = 0; p < P; p++) present[p] = FLD(T, F_ALIVE, p);

  /* 0. Env._validate_actions: deserialize against the previous observation's state */
  for (int p = 0; p < P; p++) {
    if (!present[p]) continue;
    const int32_t* a = actions + ((size_t)e * P + p) * NMMO_N_ACTION_HEADS;
    if (a[8] >= 0 && a[8] < 5) move_dir[p] = a[8];
    if (sys_on(o, NMMO_SYS_COMBAT) && a[0] >= 0 && a[0] < 3 && a[1] >= 0 && a[1] < N_OBS) {
      int nv = visible_slots(o, e, p, vis);
      if (nv > N_OBS) nv = N_OBS;
      if (a[1] < nv) { atk_t[p] = vis[a[1]]; atk_s[p] = a[0]; }
    }
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
    if (!sys_on(o, NMMO_SYS_RESOURCE)) continue;
    int org = FLD(T, F_HEALTH, s), h = org;
    if (FLD(T, F_FOOD, s) > 50 && FLD(T, F_WATER, s) > 50) h = h + 10 > 100 ? 100 : h + 10;
    int dmg = FLD(T, F_RESILIENT, s) ? 5 : 10;
    if (FLD(T, F_FOOD, s) == 0) h = h - dmg < 0 ? 0 : h - dmg;
    if (FLD(T, F_WATER, s) == 0) h = h - dmg < 0 ? 0 : h - dmg;
    FLD(T, F_HEALTH, s) = (int16_t)h;
    FLD(T, F_HEALTH_RESTORE, s) = (int16_t)(h - org);
    int r = FLD(T, F_ROW, s), c = FLD(T, F_COL, s);
    int fd = FLD(T, F_FOOD, s) - 5;
    FLD(T, F_FOOD, s) = (int16_t)(fd < 0 ? 0 : fd);
    if (mat[r * SIZE + c] == M_FOILAGE) { /* Food.update -> harvest (depletes) */
      FLD(T, F_FOOD, s) = 100;
      mat[r * SIZE + c] = M_SCRUB;
    }
    int wt = FLD(T, F_WATER, s) - 5;
    FLD(T, F_WATER, s) = (int16_t)(wt < 0 ? 0 : wt);
    if (mat[(r - 1) * SIZE + c] == M_WATER || mat[(r + 1) * SIZE + c] == M_WATER ||
        mat[r * SIZE + c - 1] == M_WATER || mat[r * SIZE + c + 1] == M_WATER)
      FLD(T, F_WATER, s) = 100;
  }
  /* 3. actions by priority: Attack (50) then Move (60), slot order */
  for (int s = 0; s < P + E[E_NPC_COUNT]; s++)
    if (atk_t[s] >= 0) attack_call(o, e, s, atk_s[s], atk_t[s]);
  for (int s = 0; s < P + E[E_NPC_COUNT]; s++)
    if (move_dir[s] >= 0) move_call(o, e, s, move_dir[s]);
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
    }
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
  /* 7. NPC refill */
  if (sys_on(o, NMMO_SYS_NPC)) npc_spawn(o, e, tick + 1);
  /* 8. rewards, dones */
  int alive = E[E_PLAYERS_ALIVE];
  int done = alive == 0 || (int)(tick + 1) >= o->cfg.horizon || alive <= o->cfg.early_stop_agent_num;
  double nt = (double)o->cfg.task_num_tick;
  double p_new = (double)(tick + 1) / nt, p_old = (double)tick / nt;
  if (p_new > 1.0) p_new = 1.0;
  if (p_old > 1.0) p_old = 1.0;
  for (int p = 0; p < P; p++) {
    size_t i = (size_t)e * P + p;
    float rw = 0.f;
    if (present[p]) rw = died[p] ? -1.f : (float)(p_new - p_old);
    if (rew) rew[i] = rw;
    if (term) term[i] = (uint8_t)died[p];
    if (trunc) trunc[i] = (uint8_t)(done && FLD(T, F_ALIVE, p));
    if (mask) mask[i] = (uint8_t)present[p];
  }
  E[E_DONE] = done;
  write_obs(o, e, obs_env);
}

/* ------------------------------------------------------------------ scripted policy (SPEC §9) */
static void scripted_env(Oracle* o, int e, uint64_t pseed, int32_t* actions) {
  const int S = o->S, P = o->P;
  const int16_t* T = ENT(o, e);
  const int32_t* E = ENV(o, e);
  const uint8_t* mat = o->mat + (size_t)e * NMMO_MAP_TILES;
  int vis[512];
  for (int p = 0; p < P; p++) {
    int32_t* a = actions + ((size_t)e * P + p) * NMMO_N_ACTION_HEADS;
    for (int h = 0; h < NMMO_N_ACTION_HEADS; h++) a[h] = 0;
    if (!FLD(T, F_ALIVE, p)) continue;
    uint32_t ctr[4] = {(uint32_t)E[E_TICK] + 2048u * (uint32_t)E[E_EPISODE],
                       (uint32_t)E[E_ENV_INDEX], (uint32_t)p, 0}, u[4];
    int r = FLD(T, F_ROW, p), c = FLD(T, F_COL, p);
    a[1] = N_OBS; a[2] = 1024; a[3] = 12; a[4] = 12; a[5] = N_OBS; a[6] = 0; a[7] = N_OBS;
    a[9] = 12; a[10] = 0; a[11] = 12;
    if (sys_on(o, NMMO_SYS_COMBAT)) {
      ctr[3] = 0;
      philox(ctr, (uint32_t)pseed, (uint32_t)(pseed >> 32), u);
      a[0] = (int32_t)U(u[0], 3);
      int nv = visible_slots(o, e, p, vis), bits[N_OBS + 1], nb = 0;
      if (nv > N_OBS) nv = N_OBS;
      for (int i = 0; i < nv; i++) {
        int s = vis[i];
        if (s != p && linf(r, c, FLD(T, F_ROW, s), FLD(T, F_COL, s)) <= 3 &&
            !(s < P && FLD(T, F_TIME_ALIVE, s) < o->cfg.spawn_immunity))
          bits[nb++] = i;
      }
      bits[nb++] = N_OBS;
      ctr[3] = 1;
      philox(ctr, (uint32_t)pseed, (uint32_t)(pseed >> 32), u);
      a[1] = bits[U(u[0], (uint32_t)nb)];
    }
    int mv[5], nm = 0;
    for (int d = 0; d < 5; d++)
      if (!impassable(mat[(r + DR[d]) * SIZE + c + DC[d]])) mv[nm++] = d;
    ctr[3] = 8;
    philox(ctr, (uint32_t)pseed, (uint32_t)(pseed >> 32), u);
    a[8] = mv[U(u[0], (uint32_t)nm)];
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
EXPORT size_t oracle_state_bytes_per_env(int slots) {
  return NMMO_NE * 4 + (size_t)NMMO_NF * slots * 2 + (size_t)slots * 2 + NMMO_MAP_TILES;
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
  for (int m = 0; m < cfg->map_n; m++)
    generate_map(cfg->map_seed, (uint32_t)m, o->bank + (size_t)m * NMMO_MAP_TILES);
  for (int k = 0; k < cfg->task_embed_dim; k++) o->task[k] = task_emb ? half_to_float(task_emb[k]) : 0.f;
  return o;
}

EXPORT void oracle_destroy(void* h) {
  Oracle* o = (Oracle*)h;
  if (!o) return;
  free(o->env); free(o->ent); free(o->ring); free(o->mat); free(o->bank); free(o);
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
  size_t per = oracle_state_bytes_per_env(o->S);
  if (nbytes != per * (size_t)o->n_envs) return NMMO_E_SIZE;
  uint8_t* b = (uint8_t*)buf;
  for (int e = 0; e < o->n_envs; e++) {
    memcpy(b, ENV(o, e), NMMO_NE * 4); b += NMMO_NE * 4;
    memcpy(b, ENT(o, e), (size_t)NMMO_NF * o->S * 2); b += (size_t)NMMO_NF * o->S * 2;
    memcpy(b, o->ring + (size_t)e * o->S, (size_t)o->S * 2); b += (size_t)o->S * 2;
    memcpy(b, o->mat + (size_t)e * NMMO_MAP_TILES, NMMO_MAP_TILES); b += NMMO_MAP_TILES;
  }
  return 0;
}
EXPORT int oracle_set_state(void* h, const void* buf, size_t nbytes) {
  Oracle* o = (Oracle*)h;
  size_t per = oracle_state_bytes_per_env(o->S);
  if (nbytes != per * (size_t)o->n_envs) return NMMO_E_SIZE;
  const uint8_t* b = (const uint8_t*)buf;
  for (int e = 0; e < o->n_envs; e++) {
    memcpy(ENV(o, e), b, NMMO_NE * 4); b += NMMO_NE * 4;
    memcpy(ENT(o, e), b, (size_t)NMMO_NF * o->S * 2); b += (size_t)NMMO_NF * o->S * 2;
    memcpy(o->ring + (size_t)e * o->S, b, (size_t)o->S * 2); b += (size_t)o->S * 2;
    memcpy(o->mat + (size_t)e * NMMO_MAP_TILES, b, NMMO_MAP_TILES); b += NMMO_MAP_TILES;
  }
  return 0;
}
EXPORT int oracle_get_map_bank(void* h, uint8_t* buf, size_t nbytes) {
  Oracle* o = (Oracle*)h;
  if (nbytes != (size_t)o->cfg.map_n * NMMO_MAP_TILES) return NMMO_E_SIZE;
  memcpy(buf, o->bank, nbytes);
  return 0;
}
