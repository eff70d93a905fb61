// tick.hip — the Realm tick (SPEC.md §4-§6) as one gfx950 workgroup per env.
//
// Replaces nmmo.Env.step / Env.reset behind the reference's call sites
// (reinforcement_learning/stat_wrapper.py:51,64; clean_pufferl.py:175,293,357).
//
// Execution model: thread s owns entity slot s (players 0..P-1, NPCs P.. in spawn order); the
// env's whole entity table (43 int16 fields x slots, ~33 KB at 384 slots), the free-row ring
// and the depleted-tile bitmap live in LDS for the duration of the tick; the material map stays
// in HBM/L2 (sparse per-entity accesses). nmmo's Python executes every phase one entity at a
// time in insertion order; each phase here is parallel over slots, and the order dependence is
// resolved exactly:
//   * food harvest: a player eats iff its tile is Foilage at phase start and no lower slot in
//     the realm stands on it (first-in-slot-order wins, later ones see Scrub);
//   * attacks: an attack is *contested* iff an earlier attack targets its attacker or its
//     target, or its target attacked earlier. Uncontested attacks read only phase-start state
//     and have disjoint write sets, so they are applied in parallel first; contested ones are
//     then replayed lane-serially in slot order (the only serial part of the tick);
//   * cull, free-row FIFO, NPC compaction and NPC spawn use wave ballots + block prefix counts.
#include "kernels.h"

namespace nmmo {

struct Ctx {
  int16_t* T;        // [kNFLive][S]
  int16_t* rowslot;  // [S+1] datastore row -> slot
  int16_t* amove;    // [S]
  int16_t* atgt;     // [S]
  int16_t* asty;     // [S]
  int* ft;           // [S] first attacker slot targeting each slot
  int16_t* clist;    // [S] contested attackers
  int16_t* ring;     // [S]
  uint32_t* dep;     // [kBitmapWords]
  int* E;            // [NMMO_NE]
  int* wtot;         // [32] wave totals
  int* misc;         // [16]
  uint8_t* pres;     // [128] present at tick start
  uint8_t* died;     // [128]
  uint8_t* mat;      // global, this env
  const uint8_t* bank;
  int S, P, N;
  const NmmoConfig* cfg;
};

#define TF(f, s) c.T[(f) * c.S + (s)]

__device__ inline bool sys(const Ctx& c, uint32_t b) { return (c.cfg->systems & b) != 0; }
__device__ inline uint64_t env_seed(const Ctx& c) {
  return (uint64_t)(uint32_t)c.E[E_SEED_LO] | ((uint64_t)(uint32_t)c.E[E_SEED_HI] << 32);
}

__host__ __device__ inline size_t tick_lds_bytes(int S) {
  auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
  size_t b = 0;
  b += al((size_t)kNFLive * S * 2);  // T
  b += al((size_t)(S + 1) * 2);      // rowslot
  b += 3 * al((size_t)S * 2);        // amove atgt asty
  b += al((size_t)S * 4);            // ft
  b += al((size_t)S * 2);            // clist
  b += al((size_t)S * 2);            // ring
  b += (size_t)kBitmapWords * 4;     // dep
  b += NMMO_NE * 4 + 32 * 4 + 16 * 4 + 128 + 128;
  return b;
}

__device__ inline Ctx make_ctx(unsigned char* smem, const DevState& st, int e) {
  auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
  Ctx c;
  const int S = st.S;
  size_t o = 0;
  c.T = reinterpret_cast<int16_t*>(smem + o); o += al((size_t)kNFLive * S * 2);
  c.rowslot = reinterpret_cast<int16_t*>(smem + o); o += al((size_t)(S + 1) * 2);
  c.amove = reinterpret_cast<int16_t*>(smem + o); o += al((size_t)S * 2);
  c.atgt = reinterpret_cast<int16_t*>(smem + o); o += al((size_t)S * 2);
  c.asty = reinterpret_cast<int16_t*>(smem + o); o += al((size_t)S * 2);
  c.ft = reinterpret_cast<int*>(smem + o); o += al((size_t)S * 4);
  c.clist = reinterpret_cast<int16_t*>(smem + o); o += al((size_t)S * 2);
  c.ring = reinterpret_cast<int16_t*>(smem + o); o += al((size_t)S * 2);
  c.dep = reinterpret_cast<uint32_t*>(smem + o); o += (size_t)kBitmapWords * 4;
  c.E = reinterpret_cast<int*>(smem + o); o += NMMO_NE * 4;
  c.wtot = reinterpret_cast<int*>(smem + o); o += 32 * 4;
  c.misc = reinterpret_cast<int*>(smem + o); o += 16 * 4;
  c.pres = smem + o; o += 128;
  c.died = smem + o; o += 128;
  c.mat = st.mat + (size_t)e * kTiles;
  c.bank = st.bank;
  c.S = S;
  c.P = st.P;
  c.N = st.N;
  c.cfg = &st.cfg;
  return c;
}

// ---------------------------------------------------------------- load / store
__device__ void load_env(Ctx& c, const DevState& st, int e) {
  const int tid = threadIdx.x, nt = blockDim.x, S = c.S;
  if (tid < NMMO_NE) c.E[tid] = st.env[(size_t)e * NMMO_NE + tid];
  const int16_t* src = st.ent + (size_t)e * NMMO_NF * S;
  const int n16 = kNFLive * S;
  if ((S & 7) == 0) {
    const uint4* s4 = reinterpret_cast<const uint4*>(src);
    uint4* d4 = reinterpret_cast<uint4*>(c.T);
    for (int i = tid; i < n16 / 8; i += nt) d4[i] = s4[i];
  } else {
    for (int i = tid; i < n16; i += nt) c.T[i] = src[i];
  }
  for (int i = tid; i < S; i += nt) c.ring[i] = st.ring[(size_t)e * S + i];
  for (int i = tid; i < kBitmapWords; i += nt) c.dep[i] = st.dep[(size_t)e * kBitmapWords + i];
}

__device__ void store_env(const Ctx& c, const DevState& st, int e) {
  const int tid = threadIdx.x, nt = blockDim.x, S = c.S;
  if (tid < NMMO_NE) st.env[(size_t)e * NMMO_NE + tid] = c.E[tid];
  int16_t* dst = st.ent + (size_t)e * NMMO_NF * S;
  const int n16 = kNFLive * S;
  if ((S & 7) == 0) {
    const uint4* s4 = reinterpret_cast<const uint4*>(c.T);
    uint4* d4 = reinterpret_cast<uint4*>(dst);
    for (int i = tid; i < n16 / 8; i += nt) d4[i] = s4[i];
  } else {
    for (int i = tid; i < n16; i += nt) dst[i] = c.T[i];
  }
  for (int i = tid; i < S; i += nt) st.ring[(size_t)e * S + i] = c.ring[i];
  for (int i = tid; i < kBitmapWords; i += nt) st.dep[(size_t)e * kBitmapWords + i] = c.dep[i];
}

// ---------------------------------------------------------------- NPC spawn (SPEC §5.7)
// 25 attempts evaluated by lanes 0..24 of wave 0; accepted in attempt order up to capacity.
__device__ void npc_spawn(Ctx& c, uint32_t tick) {
  if (wave_id() == 0) {
    const int a = lane_id();
    const uint64_t seed = env_seed(c);
    bool valid = false;
    int r = 0, col = 0, type = 0, style = 0, level = 0;
    if (a < 25) {
      const U4 u = draw(seed, tick, P_NPC_SPAWN, (uint32_t)a, 0);
      r = kLo + (int)uniform_n(u.x, kCenter);
      col = kLo + (int)uniform_n(u.y, kCenter);
      valid = !impassable(c.mat[r * kSize + col]);
      int dist = r - kLo;
      dist = min(dist, kHi - r);
      dist = min(dist, col - kLo);
      dist = min(dist, kHi - col);
      type = 20 * dist >= 1024 ? 3 : 20 * dist >= 640 ? 2 : 1;
      style = (int)uniform_n(u.z, 3);
      level = sys(c, NMMO_SYS_PROGRESSION) ? (9 * dist) / 64 + 1 : 0;
    }
    const uint64_t b = __ballot(valid);
    const int rank = __popcll(b & lanes_below());
    const int cnt = c.E[E_NPC_COUNT], room = c.N - cnt, head = c.E[E_FREE_HEAD];
    const int nacc = min(__popcll(b), room);
    if (valid && rank < room) {
      const int s = c.P + cnt + rank;
      for (int f = 0; f < kNFLive; f++) TF(f, s) = 0;
      TF(F_ID, s) = (int16_t)(c.E[E_NPC_NEXT_ID] - rank);
      TF(F_NPC_TYPE, s) = (int16_t)type;
      TF(F_ROW, s) = (int16_t)r;
      TF(F_COL, s) = (int16_t)col;
      TF(F_HEALTH, s) = 100;
      TF(F_FOOD, s) = 100;
      TF(F_WATER, s) = 100;
      TF(F_MELEE_LEVEL, s) = 1;
      TF(F_RANGE_LEVEL, s) = 1;
      TF(F_MAGE_LEVEL, s) = 1;
      if (level > 0) {
        TF(F_MELEE_LEVEL + 2 * style, s) = (int16_t)level;
        TF(F_MELEE_EXP + 2 * style, s) = (int16_t)exp_at_level(level);
      }
      if (sys(c, NMMO_SYS_EXCHANGE)) TF(F_GOLD, s) = (int16_t)level;
      TF(F_ALIVE, s) = 1;
      TF(F_DS_ROW, s) = c.ring[(head + rank) % c.S];
      TF(F_STYLE, s) = (int16_t)style;
      TF(F_NPC_LEVEL, s) = (int16_t)level;
    }
    if (lane_id() == 0 && nacc > 0) {
      c.E[E_FREE_HEAD] = (head + nacc) % c.S;
      c.E[E_FREE_COUNT] -= nacc;
      c.E[E_NPC_NEXT_ID] -= nacc;
      c.E[E_NPC_COUNT] = cnt + nacc;
    }
  }
  __syncthreads();
}

// ---------------------------------------------------------------- reset (SPEC §4)
__device__ void reset_env(Ctx& c, uint64_t seed, int episode, int env_global) {
  const int tid = threadIdx.x, nt = blockDim.x, S = c.S, P = c.P;
  for (int i = tid; i < kNFLive * S; i += nt) c.T[i] = 0;
  for (int i = tid; i < kBitmapWords; i += nt) c.dep[i] = 0;
  for (int i = tid; i < S; i += nt) c.ring[i] = i < c.N ? (int16_t)(P + 1 + i) : (int16_t)0;
  if (tid < NMMO_NE) c.E[tid] = 0;
  __syncthreads();
  if (tid == 0) {
    c.E[E_SEED_LO] = (int)(uint32_t)seed;
    c.E[E_SEED_HI] = (int)(uint32_t)(seed >> 32);
    c.E[E_EPISODE] = episode;
    c.E[E_ENV_INDEX] = env_global;
    c.E[E_MAP_ID] = (int)uniform_n(draw(seed, 0, P_MAPSEL, 0, 0).x, (uint32_t)c.cfg->map_n);
    c.E[E_FREE_COUNT] = c.N;
    c.E[E_NPC_NEXT_ID] = -1;
    c.E[E_PLAYERS_ALIVE] = P;
  }
  __syncthreads();
  {  // copy the bank map into the env's mutable map (16 B per lane)
    const uint4* src = reinterpret_cast<const uint4*>(c.bank + (size_t)c.E[E_MAP_ID] * kTiles);
    uint4* dst = reinterpret_cast<uint4*>(c.mat);
    for (int i = tid; i < kTiles / 16; i += nt) dst[i] = src[i];
  }
  if (tid < P) {
    const uint32_t off = uniform_n(draw(seed, 0, P_SPAWN_OFFSET, 0, 0).x, 508);
    const uint32_t p = (off + (uint32_t)(tid * 508 / P)) % 508, side = p / 127, k = p % 127;
    const int r = side == 0 ? kLo : side == 1 ? kLo + (int)k : side == 2 ? kHi : kHi - (int)k;
    const int col = side == 0 ? kLo + (int)k : side == 1 ? kHi : side == 2 ? kHi - (int)k : kLo;
    const uint32_t u = draw(seed, 0, P_RESILIENT, (uint32_t)tid, 0).x;
    TF(F_ID, tid) = (int16_t)(tid + 1);
    TF(F_ROW, tid) = (int16_t)r;
    TF(F_COL, tid) = (int16_t)col;
    TF(F_HEALTH, tid) = 100;
    TF(F_FOOD, tid) = 100;
    TF(F_WATER, tid) = 100;
#pragma unroll
    for (int sk = 0; sk < 8; sk++) TF(F_MELEE_LEVEL + 2 * sk, tid) = 1;
    TF(F_ALIVE, tid) = 1;
    TF(F_DS_ROW, tid) = (int16_t)(tid + 1);
    TF(F_RESILIENT, tid) = u < c.cfg->resilient_u32 ? 1 : 0;
  }
  __syncthreads();
  if (sys(c, NMMO_SYS_NPC)) npc_spawn(c, 0);
}

// ---------------------------------------------------------------- NPC AI (SPEC §6)
__device__ inline bool player_valid(const Ctx& c, int id, int r, int col) {
  if (id <= 0 || id > c.P) return false;
  const int s = id - 1;
  return TF(F_ALIVE, s) && TF(F_HEALTH, s) > 0 && linf(r, col, TF(F_ROW, s), TF(F_COL, s)) <= kVision;
}

__device__ void npc_decide(Ctx& c, int n, int& move, int& tgt, int& sty) {
  const int r = TF(F_ROW, n), col = TF(F_COL, n), id = TF(F_ID, n);
  const U4 u = draw(env_seed(c), (uint32_t)c.E[E_TICK], P_NPC_MOVE, (uint32_t)(-id), 0);
  move = -1;
  tgt = -1;
  sty = TF(F_STYLE, n);
  if (!player_valid(c, TF(F_ATTACKER_ID, n), r, col)) TF(F_ATTACKER_ID, n) = 0;
  if (!player_valid(c, TF(F_TARGET_ID, n), r, col)) TF(F_TARGET_ID, n) = 0;
  const int type = TF(F_NPC_TYPE, n);
  bool hunt = false;
  if (type == 2 && TF(F_ATTACKER_ID, n)) {
    TF(F_TARGET_ID, n) = TF(F_ATTACKER_ID, n);
    hunt = true;
  } else if (type == 3) {
    if (!TF(F_TARGET_ID, n)) {
      int best = -1, bd = 1 << 30;
      for (int p = 0; p < c.P; p++) {
        if (!TF(F_ALIVE, p) || TF(F_HEALTH, p) <= 0) continue;
        const int d = linf(r, col, TF(F_ROW, p), TF(F_COL, p));
        if (d <= kVision && d < bd) { bd = d; best = p; }
      }
      if (best >= 0) TF(F_TARGET_ID, n) = TF(F_ID, best);
    }
    hunt = TF(F_TARGET_ID, n) != 0;
  }
  if (!hunt) {
    int cand[4], k = 0;
#pragma unroll
    for (int d = 0; d < 4; d++)
      if (!impassable(c.mat[(r + dir_dr(d)) * kSize + col + dir_dc(d)])) cand[k++] = d;
    if (k) move = cand[uniform_n(u.x, (uint32_t)k)];
    return;
  }
  const int ts = TF(F_TARGET_ID, n) - 1;
  const int tr = TF(F_ROW, ts), tc = TF(F_COL, ts);
  const int dist = linf(r, col, tr, tc);
  if (dist == 0) {
    move = (int)uniform_n(u.y, 4);
  } else if (dist > 1) {
    const int dr = tr - r, dc = tc - col;
    const int dir_r = dr > 0 ? 1 : 0, dir_c = dc > 0 ? 2 : 3;
    const bool rows_first = iabs(dr) >= iabs(dc);
    const int first = rows_first ? dir_r : dir_c, second = rows_first ? dir_c : dir_r;
    const bool second_nz = rows_first ? dc != 0 : dr != 0;
    if (!impassable(c.mat[(r + dir_dr(first)) * kSize + col + dir_dc(first)])) move = first;
    else if (second_nz && !impassable(c.mat[(r + dir_dr(second)) * kSize + col + dir_dc(second)]))
      move = second;
  }
  if (dist <= 3) tgt = ts;
}

// ---------------------------------------------------------------- combat (SPEC §5.3)
__device__ inline int combat_level(const Ctx& c, int s) {
  const int nsk = s < c.P ? 8 : 3;
  int l = 0;
  for (int k = 0; k < nsk; k++) l = max(l, (int)TF(F_MELEE_LEVEL + 2 * k, s));
  return l;
}

// Attack.call validity + combat.attack damage on the current LDS state; -1 = no attack.
__device__ int eval_attack(const Ctx& c, int x, int sty, int t) {
  if (!TF(F_ALIVE, x) || TF(F_HEALTH, x) <= 0) return -1;
  if (!TF(F_ALIVE, t) || TF(F_HEALTH, t) <= 0 || t == x) return -1;
  if (x < c.P && t < c.P && TF(F_TIME_ALIVE, t) < c.cfg->spawn_immunity) return -1;
  if (x >= c.P && t >= c.P) return -1;
  if (linf(TF(F_ROW, x), TF(F_COL, x), TF(F_ROW, t), TF(F_COL, t)) > 3) return -1;
  const bool prog = sys(c, NMMO_SYS_PROGRESSION);
  int offense = prog ? 10 + 5 * TF(F_MELEE_LEVEL + 2 * sty, x) : 30;
  int defense = prog ? 5 * combat_level(c, t) : 0;
  if (sys(c, NMMO_SYS_EQUIPMENT)) {
    offense += TF(F_EQUIP_OFFENSE, x);
    defense += TF(F_EQUIP_DEFENSE, t);
  }
  const int e0 = TF(F_MELEE_EXP, t), e1 = TF(F_RANGE_EXP, t), e2 = TF(F_MAGE_EXP, t);
  const int mx = max(e0, max(e1, e2)), mn = min(e0, min(e1, e2));
  int mult4 = 4;
  if (mx != mn) {
    const int dom = e0 == mx ? 0 : e1 == mx ? 1 : 2;
    const int weak = dom == 0 ? 2 : dom == 1 ? 0 : 1;  // melee<-mage, range<-melee, mage<-range
    if (sty == weak) mult4 = 6;
  }
  const int d4 = max(mult4 * offense - 4 * defense, offense);
  return d4 >> 2;
}

__device__ void apply_attack(Ctx& c, int x, int sty, int t, int dmg, int tick) {
  TF(F_ATTACKER_ID, t) = TF(F_ID, x);
  if (x < c.P && sys(c, NMMO_SYS_PROGRESSION)) {
    const int f = F_MELEE_EXP + 2 * sty;
    const int ex = TF(f, x) + 6;
    TF(f, x) = (int16_t)ex;
    const int nl = level_at_exp(ex);
    if (nl > TF(f - 1, x)) TF(f - 1, x) = (int16_t)nl;
  }
  TF(F_DAMAGE, t) = (int16_t)dmg;
  const int h = max(0, (int)TF(F_HEALTH, t) - dmg);
  TF(F_HEALTH, t) = (int16_t)h;
  if (h == 0) TF(F_PLAYER_KILLS, x) += 1;
  TF(F_LATEST_COMBAT_TICK, x) = (int16_t)(tick + 1);
  TF(F_LATEST_COMBAT_TICK, t) = (int16_t)(tick + 1);
}

// ---------------------------------------------------------------- the tick (SPEC §5)
__device__ void tick_env(Ctx& c, const int32_t* __restrict__ act, float* rew, uint8_t* term,
                         uint8_t* trunc, uint8_t* mask) {
  const int tid = threadIdx.x, nt = blockDim.x, S = c.S, P = c.P;
  const int s = tid;
  const int tick = c.E[E_TICK];
  const int nslots = P + c.E[E_NPC_COUNT];
  const bool inslot = s < nslots;

  if (s < P) c.pres[s] = (uint8_t)TF(F_ALIVE, s);
  for (int k = tid; k <= S; k += nt) c.rowslot[k] = -1;
  __syncthreads();
  if (inslot && TF(F_ALIVE, s)) c.rowslot[TF(F_DS_ROW, s)] = (int16_t)s;
  __syncthreads();

  // 0. decode (Env._validate_actions) against the previous observation's state
  int my_move = -1, my_tgt = -1, my_sty = 0;
  if (s < P && c.pres[s]) {
    const int32_t* a = act + (size_t)s * kHeads;
    const int dmove = a[8], dsty = a[0], dk = a[1];
    if (dmove >= 0 && dmove < 5) my_move = dmove;
    if (sys(c, NMMO_SYS_COMBAT) && dsty >= 0 && dsty < 3 && dk >= 0 && dk < kNObs) {
      const int r = TF(F_ROW, s), col = TF(F_COL, s);
      int cnt = 0;
      for (int row = 1; row <= S && cnt <= dk; row++) {
        const int q = c.rowslot[row];
        if (q < 0 || linf(r, col, TF(F_ROW, q), TF(F_COL, q)) > kVision) continue;
        if (cnt == dk) { my_tgt = q; my_sty = dsty; }
        cnt++;
      }
    }
  }
  // 1. npcs.actions
  if (sys(c, NMMO_SYS_NPC) && s >= P && inslot) npc_decide(c, s, my_move, my_tgt, my_sty);
  if (s < S) {
    c.amove[s] = (int16_t)my_move;
    c.atgt[s] = (int16_t)my_tgt;
    c.asty[s] = (int16_t)my_sty;
  }
  __syncthreads();

  // 2. players.update / npcs.update
  bool eat = false;
  int tile = 0;
  if (inslot && TF(F_ALIVE, s)) {
    if (TF(F_DAMAGE, s) == 0) TF(F_ATTACKER_ID, s) = 0;
    TF(F_DAMAGE, s) = 0;
    TF(F_TIME_ALIVE, s) += 1;
    if (s >= P) {
      TF(F_HEALTH, s) = (int16_t)min(100, TF(F_HEALTH, s) + 1);
    } else if (sys(c, NMMO_SYS_RESOURCE)) {
      const int org = TF(F_HEALTH, s);
      int h = org;
      const int food = TF(F_FOOD, s), water = TF(F_WATER, s);
      if (food > 50 && water > 50) h = min(100, h + 10);
      const int dmg = TF(F_RESILIENT, s) ? 5 : 10;
      if (food == 0) h = max(0, h - dmg);
      if (water == 0) h = max(0, h - dmg);
      TF(F_HEALTH, s) = (int16_t)h;
      TF(F_HEALTH_RESTORE, s) = (int16_t)(h - org);
      TF(F_FOOD, s) = (int16_t)max(0, food - 5);
      const int r = TF(F_ROW, s), col = TF(F_COL, s);
      tile = r * kSize + col;
      eat = c.mat[tile] == M_FOILAGE;
      for (int q = 0; q < s && eat; q++)  // first player in slot order on the tile wins
        if (TF(F_ALIVE, q) && TF(F_ROW, q) == r && TF(F_COL, q) == col) eat = false;
      const bool drink = c.mat[tile - kSize] == M_WATER || c.mat[tile + kSize] == M_WATER ||
                         c.mat[tile - 1] == M_WATER || c.mat[tile + 1] == M_WATER;
      TF(F_WATER, s) = (int16_t)(drink ? 100 : max(0, water - 5));
    }
  }
  __syncthreads();
  if (eat) {
    TF(F_FOOD, s) = 100;
    c.mat[tile] = M_SCRUB;
    atomicOr(&c.dep[tile >> 5], 1u << (tile & 31));
  }

  // 3a. Attack (priority 50)
  for (int k = tid; k < S; k += nt) c.ft[k] = 0x7FFF;
  __syncthreads();
  const int t = s < S ? c.atgt[s] : -1;
  const bool ev = inslot && t >= 0;
  if (ev) atomicMin(&c.ft[t], s);
  __syncthreads();
  const bool contested = ev && (c.ft[s] < s || c.ft[t] < s || (c.atgt[t] >= 0 && t < s));
  int dmg = -1;
  if (ev && !contested) dmg = eval_attack(c, s, c.asty[s], t);
  __syncthreads();
  if (dmg >= 0) apply_attack(c, s, c.asty[s], t, dmg, tick);
  int ncont;
  const int cpos = block_prefix_count(contested, c.wtot, &ncont);
  if (contested) c.clist[cpos] = (int16_t)s;
  __syncthreads();
  if (tid == 0) {  // the lane-serial replay of the contested attacks, in slot order
    for (int i = 0; i < ncont; i++) {
      const int x = c.clist[i], tx = c.atgt[x], sx = c.asty[x];
      const int d = eval_attack(c, x, sx, tx);
      if (d >= 0) apply_attack(c, x, sx, tx, d, tick);
    }
  }
  __syncthreads();

  // 3b. Move (priority 60)
  if (inslot && c.amove[s] >= 0 && TF(F_ALIVE, s) && TF(F_HEALTH, s) > 0) {
    const int d = c.amove[s];
    const int nr = TF(F_ROW, s) + dir_dr(d), nc = TF(F_COL, s) + dir_dc(d);
    if (!impassable(c.mat[nr * kSize + nc]) && TF(F_FREEZE, s) <= 0) {
      TF(F_ROW, s) = (int16_t)nr;
      TF(F_COL, s) = (int16_t)nc;
      const int progress = 64 - linf(80, 80, nr, nc);
      if (progress > TF(F_EXPLORATION, s)) TF(F_EXPLORATION, s) = (int16_t)progress;
    }
  }
  __syncthreads();

  // 4. cull: rows appended to the free ring in slot order; NPC slots compacted
  const bool dead = inslot && TF(F_ALIVE, s) && TF(F_HEALTH, s) <= 0;
  int ndead;
  const int dpos = block_prefix_count(dead, c.wtot, &ndead);
  int npdead;
  block_prefix_count(dead && s < P, c.wtot, &npdead);
  if (s < P) c.died[s] = dead ? 1 : 0;
  if (dead) {
    c.ring[(c.E[E_FREE_HEAD] + c.E[E_FREE_COUNT] + dpos) % S] = TF(F_DS_ROW, s);
    TF(F_ALIVE, s) = 0;
    if (s < P) TF(F_DIED_TICK, s) = (int16_t)(tick + 1);
  }
  __syncthreads();
  if (tid == 0) {
    c.E[E_FREE_COUNT] += ndead;
    c.E[E_PLAYERS_ALIVE] -= npdead;
  }
  if (sys(c, NMMO_SYS_NPC)) {
    const bool keep = s >= P && inslot && TF(F_ALIVE, s);
    int nkeep;
    const int kpos = block_prefix_count(keep, c.wtot, &nkeep);
    int16_t v[kNFLive];
    if (keep) {
#pragma unroll
      for (int f = 0; f < kNFLive; f++) v[f] = TF(f, s);
    }
    __syncthreads();
    if (keep) {
#pragma unroll
      for (int f = 0; f < kNFLive; f++) TF(f, P + kpos) = v[f];
    }
    if (s >= P + nkeep && inslot) {
#pragma unroll
      for (int f = 0; f < kNFLive; f++) TF(f, s) = 0;
    }
    if (tid == 0) c.E[E_NPC_COUNT] = nkeep;
  }
  __syncthreads();

  // 5-6. tick += 1; map.step respawn of depleted tiles
  const uint64_t seed = env_seed(c);
  {
    const uint8_t* base = c.bank + (size_t)c.E[E_MAP_ID] * kTiles;
    for (int w = tid; w < kBitmapWords; w += nt) {
      uint32_t bits = c.dep[w], keepb = bits;
      while (bits) {
        const int b = __builtin_ctz(bits);
        bits &= bits - 1;
        const int tt = w * 32 + b;
        const int bm = base[tt];
        if (draw(seed, (uint32_t)(tick + 1), P_RESPAWN, (uint32_t)tt, 0).x < respawn_u32(bm)) {
          c.mat[tt] = (uint8_t)bm;
          keepb &= ~(1u << b);
        }
      }
      c.dep[w] = keepb;
    }
  }
  __syncthreads();
  if (tid == 0) c.E[E_TICK] = tick + 1;
  __syncthreads();
  // 7. NPC refill
  if (sys(c, NMMO_SYS_NPC)) npc_spawn(c, (uint32_t)(tick + 1));

  // 8. rewards / dones
  if (tid == 0) {
    const int alive = c.E[E_PLAYERS_ALIVE];
    const int done = alive == 0 || tick + 1 >= c.cfg->horizon || alive <= c.cfg->early_stop_agent_num;
    c.E[E_DONE] = done;
  }
  __syncthreads();
  if (s < P) {
    const double nt_ = (double)c.cfg->task_num_tick;
    const double pn = fmin((double)(tick + 1) / nt_, 1.0), po = fmin((double)tick / nt_, 1.0);
    float rw = 0.f;
    if (c.pres[s]) rw = c.died[s] ? -1.f : (float)(pn - po);
    rew[s] = rw;
    term[s] = c.died[s];
    trunc[s] = (uint8_t)(c.E[E_DONE] && TF(F_ALIVE, s));
    mask[s] = c.pres[s];
  }
}

// ---------------------------------------------------------------- kernel
// mode 0: step (auto-reset envs that are done); mode 1: reset every env.
__global__ void tick_kernel(DevState st, const int32_t* __restrict__ actions,
                            const uint64_t* __restrict__ env_seeds, float* rew, uint8_t* term,
                            uint8_t* trunc, uint8_t* mask, int mode) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int e = blockIdx.x;
  Ctx c = make_ctx(smem, st, e);
  load_env(c, st, e);
  __syncthreads();
  const size_t o = (size_t)e * c.P;
  if (mode == 1 || c.E[E_DONE]) {
    const int env_global = (int)(st.cfg.env_index_base + (uint64_t)e);
    uint64_t seed;
    int episode;
    if (mode == 1) {
      seed = env_seeds ? env_seeds[e] : splitmix64(st.seed ^ splitmix64((uint64_t)env_global));
      episode = 0;
    } else {
      seed = splitmix64(env_seed(c) ^ (0xD1B54A32D192ED03ull * (uint64_t)(c.E[E_EPISODE] + 1)));
      episode = c.E[E_EPISODE] + 1;
    }
    __syncthreads();
    reset_env(c, seed, episode, env_global);
    for (int p = threadIdx.x; p < c.P; p += blockDim.x) {
      if (rew) rew[o + p] = 0.f;
      if (term) term[o + p] = 0;
      if (trunc) trunc[o + p] = 0;
      if (mask) mask[o + p] = 1;
    }
  } else {
    tick_env(c, actions + o * kHeads, rew + o, term + o, trunc + o, mask + o);
  }
  __syncthreads();
  store_env(c, st, e);
}

hipError_t launch_tick(const DevState& st, const int32_t* actions, const uint64_t* env_seeds,
                       float* rew, uint8_t* term, uint8_t* trunc, uint8_t* mask, int mode,
                       hipStream_t stream) {
  const int threads = ((st.S + 63) / 64) * 64;
  hipLaunchKernelGGL(tick_kernel, dim3(st.n_envs), dim3(threads), tick_lds_bytes(st.S), stream,
                     st, actions, env_seeds, rew, term, trunc, mask, mode);
  return hipGetLastError();
}

// set_state support: the depleted-tile bitmap is derived state (bit <=> material != bank).
__global__ void rebuild_dep_kernel(DevState st) {
  const int e = blockIdx.x;
  const int32_t* E = st.env + (size_t)e * NMMO_NE;
  const uint8_t* mat = st.mat + (size_t)e * kTiles;
  const uint8_t* base = st.bank + (size_t)E[E_MAP_ID] * kTiles;
  for (int w = threadIdx.x; w < kBitmapWords; w += blockDim.x) {
    uint32_t bits = 0;
    for (int b = 0; b < 32; b++) bits |= (mat[w * 32 + b] != base[w * 32 + b] ? 1u : 0u) << b;
    st.dep[(size_t)e * kBitmapWords + w] = bits;
  }
}

hipError_t launch_rebuild_dep(const DevState& st, hipStream_t stream) {
  hipLaunchKernelGGL(rebuild_dep_kernel, dim3(st.n_envs), dim3(256), 0, stream, st);
  return hipGetLastError();
}

}  // namespace nmmo
