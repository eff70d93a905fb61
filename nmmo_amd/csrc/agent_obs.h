// agent_obs.h — the per-agent observation pieces shared by the native (SPEC.md §8b,
// native_obs.hip) and wire (SPEC §8c, wire_obs.hip) obs kernels.
//
// Per workgroup (env e, kAoAgents agents; kAoWaves waves, one agent per wave at a time):
//  - ao_stage: the env's 31 Entity columns in LDS with an odd dword stride (a lane per field
//    reads one slot's row conflict-free; the field-major stride of S = 384 puts all 31 fields of
//    a slot in one bank) and one packed word per datastore row: row | slot[0:8] << 8 | col << 16
//    | slot[8] << 24 | spawn-immune << 25 | dangerous << 26 | player << 27 (kAoEmpty = no entity
//    on that row: row = col = 255, outside every window);
//  - every lane keeps the packed words of its kAoRows datastore rows in registers, so an agent's
//    window compaction (Entity.Query.window order) is kAoRows ballots with no LDS read, each row
//    tested with 16-bit packed math (row and col in the word's two halves);
//  - the ActionTargets sections are wave-uniform bit fields (ballots over the visible rows and the
//    12 inventory slots, closed forms for Style / GoldPrice / Move / SellPrice) placed into a bit
//    image with compile-time shifts (the sections' sizes are nmmo_layout's fixed dims).
#pragma once

#include <utility>

#include "kernels.h"
#include "wire.h"

namespace nmmo {

#ifndef NMMO_AO_WAVES  // (A/B builds of the native kernel's workgroup shape: tools/debug/ab_native.sh)
#define NMMO_AO_WAVES 4
#define NMMO_AO_AGENTS 16
#endif
constexpr int kAoWaves = NMMO_AO_WAVES;
constexpr int kAoAgents = NMMO_AO_AGENTS;  // agents per workgroup
constexpr int kAoRows = kMaxSlots / 64;   // packed datastore-row words per lane
constexpr uint32_t kAoEmpty = 0xFFFFFFFFu;
static_assert(kSize <= 256 && kMaxSlots <= 2 * 256 && kMaxSlots % 64 == 0, "packed entity word; two slots per thread (>= 256 threads)");
__host__ __device__ inline int ao_stride(int S) { return ((S + 1) >> 1 | 1) << 1; }  // int16, odd dword count
__host__ __device__ inline size_t ao_entity_lds(int S) {  // T | pk
  return (((size_t)NMMO_N_ENTITY_COLS * ao_stride(S) * 2 + 15) & ~(size_t)15) + (size_t)(kMaxSlots + 64) * 4;
}
__host__ __device__ inline uint32_t ao_pack(int slot, int row, int col, bool immune, bool danger, bool player) {
  return (uint32_t)(row & 255) | (uint32_t)(slot & 255) << 8 | (uint32_t)(col & 255) << 16 | (uint32_t)(slot >> 8) << 24 |
         (immune ? 1u << 25 : 0u) | (danger ? 1u << 26 : 0u) | (player ? 1u << 27 : 0u);
}
__device__ __forceinline__ int ao_slot(uint32_t w) { return (int)(((w >> 8) & 255u) | ((w >> 16) & 256u)); }
__device__ __forceinline__ int ao_row(uint32_t w) { return (int)(w & 255u); }
__device__ __forceinline__ int ao_col(uint32_t w) { return (int)((w >> 16) & 255u); }
__device__ __forceinline__ bool ao_immune(uint32_t w) { return (w >> 25) & 1u; }
__device__ __forceinline__ bool ao_danger(uint32_t w) { return (w >> 26) & 1u; }
__device__ __forceinline__ bool ao_player(uint32_t w) { return (w >> 27) & 1u; }
// L-inf distance of w's tile to (r, c) <= kVision, with rc = r | c << 16: both 16-bit halves of
// (tile - (r, c)) + kVision in 0..2 kVision
typedef unsigned short ao_u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ bool ao_in_window(uint32_t w, uint32_t rc) {
  ao_u16x2 d = __builtin_bit_cast(ao_u16x2, w & 0x00FF00FFu) - __builtin_bit_cast(ao_u16x2, rc) +
               (ao_u16x2){(unsigned short)kVision, (unsigned short)kVision};
  return (d.x > d.y ? d.x : d.y) <= 2 * kVision;
}
static_assert(kMaxSlots <= 512 && kSize <= 255, "packed entity word");

// The 12 ActionTargets sections (nmmo_layout's dims, flat order) and their flat entry offsets
// (sec_wire: offsets with Buy.MarketItem left out). Launchers check a handle's layout against
// sec_flat.
constexpr int kSecN[12] = {3, 101, NMMO_MARKET_ROWS + 1, kInv + 1, kInv + 1, kNObs + 1, 99, kNObs + 1, 5, kInv + 1, 99, kInv + 1};
__host__ __device__ constexpr int sec_flat(int k) { return k == 0 ? 0 : sec_flat(k - 1) + kSecN[k - 1]; }
__host__ __device__ constexpr int sec_wire(int k) { return k < 2 ? sec_flat(k) : sec_flat(k) - kWireBuyN; }
static_assert(sec_flat(2) == kWireBuyLo && sec_flat(12) == kMaskN && sec_flat(1) == kMkAttackT &&
                  sec_flat(3) == kMkDestroy && sec_flat(4) == kMkGiveI && sec_flat(5) == kMkGiveT &&
                  sec_flat(6) == kMkGoldP && sec_flat(7) == kMkGoldT && sec_flat(8) == kMkMove &&
                  sec_flat(9) == kMkSellI && sec_flat(10) == kMkSellP && sec_flat(11) == kMkUse,
              "sections (wire.h)");
__host__ inline bool ao_layout_ok(const ObsParams& p) {
  const int offs[12] = {p.o_style, p.o_target, p.o_buy, p.o_destroy, p.o_give_item, p.o_give_target,
                        p.o_gg_price, p.o_gg_target, p.o_move, p.o_sell_item, p.o_sell_price, p.o_use};
  for (int k = 0; k < 12; k++)
    if (offs[k] != sec_flat(k)) return false;
  return p.o_agent_id == sec_flat(12);
}

// The lane index, opaque to the optimiser: per-lane predicates built from it are recomputed where
// they are used instead of hoisted out of the agent loops as lane masks (an SGPR pair each), which
// the loops then spilled to VGPR lanes and reloaded (two v_readlane each).
__device__ __forceinline__ int ao_lane() {
  int l = (int)(threadIdx.x & 63u);
  asm volatile("" : "+v"(l));
  return l;
}

__device__ __forceinline__ uint64_t low_bits(int n) { return n >= 64 ? ~0ull : n <= 0 ? 0ull : (1ull << n) - 1ull; }
// x with lane L's value replaced by the wave-uniform v: one v_writelane_b32 (the value pinned to
// an SGPR, the lane an inline constant; this compiler has no writelane builtin)
template <int L>
__device__ __forceinline__ int writelane(int v, int x) {
  static_assert(L >= 0 && L < 64, "lane");
  int sv = __builtin_amdgcn_readfirstlane(v);
  asm volatile("" : "+s"(sv));
  asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(x) : "s"(sv), "n"(L));
  return x;
}
template <int kLane0, int kIdx0, int... D>
__device__ __forceinline__ int writelanes_(const uint32_t* img, int x, std::integer_sequence<int, D...>) {
  ((x = writelane<kLane0 + D>((int)img[kIdx0 + D], x)), ...);
  return x;
}
// lanes kLane0 .. kLane0 + kN - 1 of x take img[kIdx0 ..] (wave-uniform words)
template <int kLane0, int kIdx0, int kN>
__device__ __forceinline__ int writelanes(const uint32_t* img, int x) {
  return writelanes_<kLane0, kIdx0>(img, x, std::make_integer_sequence<int, kN>{});
}

// OR the kN-bit field lo | hi << 64 (bits >= kN zero) into img at bit kOff
template <int kOff, int kN, int kW>
__device__ __forceinline__ void put_field(uint32_t (&img)[kW], uint64_t lo, uint64_t hi) {
  static_assert((kOff + kN + 31) / 32 <= kW, "image size");
#pragma unroll
  for (int d = kOff / 32; d <= (kOff + kN - 1) / 32; d++) {
    const int st = 32 * d - kOff;  // field bit on the dword's bit 0
    uint32_t x;
    if (st < 0) x = (uint32_t)(lo << (-st));
    else if (st == 0) x = (uint32_t)lo;
    else if (st < 64) x = (uint32_t)((lo >> st) | (hi << (64 - st)));
    else x = (uint32_t)(hi >> (st - 64));
    img[d] |= x;
  }
}

// Block prologue, in two parts so a kernel can issue its other independent loads between them:
// ao_stage_load issues the loads (the Entity columns, alive / datastore row of slots tid and
// tid + blockDim, the listing count and listing tid's mlist word), ao_stage_store writes LDS
// (every thread; two barriers inside): T[f * ao_stride(S) + s] = field f (< 31) of slot s,
// pk[row - 1] = the packed word of datastore row `row` (kAoEmpty where none).
// Every load of the thread is in flight before the first LDS write: a load -> write loop waited
// one memory round trip per 16-B word (6 per thread at S = 384, blockDim 256), and the listings'
// count -> mlist -> item chain ahead of the stage was three more.
constexpr int kAoStageIt = (NMMO_N_ENTITY_COLS * (kMaxSlots / 8) + 255) / 256;
struct AoStage {
  uint4 x[kAoStageIt];
  int al[2], ds[2];
  int nm, mv;  // the env's listing count (as stored) and listing tid's mlist word (any when >= nm)
};
__device__ __forceinline__ void ao_stage_load(const ObsParams& p, int e, AoStage& r) {
  const int S = p.S, tid = threadIdx.x;
  const int16_t* E = p.ent + (size_t)e * NMMO_NF * S;
  const int w4 = S / 8;  // 16-B words per field (S % 8 == 0: checked by the launchers)
  const int nw = NMMO_N_ENTITY_COLS * w4;
  r.nm = p.mcount[e];
  r.mv = p.mlist[(size_t)e * NMMO_MARKET_ROWS + min(tid, NMMO_MARKET_ROWS - 1)];
#pragma unroll
  for (int k = 0; k < kAoStageIt; k++) {
    const int i = tid + (int)blockDim.x * k;
    const int f = i / w4, j = i - f * w4;
    r.x[k] = i < nw ? reinterpret_cast<const uint4*>(E + (size_t)f * S)[j] : make_uint4(0u, 0u, 0u, 0u);
  }
#pragma unroll
  for (int u = 0; u < 2; u++) {  // (a clamped slot: a conditional load is waited on at its branch's join)
    const int s = min(tid + (int)blockDim.x * u, S - 1);
    r.al[u] = E[F_ALIVE * S + s];
    r.ds[u] = E[F_DS_ROW * S + s];
  }
}
__device__ __forceinline__ void ao_stage_store(const ObsParams& p, int e, int16_t* T, uint32_t* pk, const AoStage& r) {
  const int S = p.S, P = p.P, Sp = ao_stride(S), tid = threadIdx.x;
  const int16_t* E = p.ent + (size_t)e * NMMO_NF * S;
  const int w4 = S / 8;
  const int nw = NMMO_N_ENTITY_COLS * w4;
  constexpr int kIt = kAoStageIt;
  const int(&al)[2] = r.al;
  const int(&ds)[2] = r.ds;
#pragma unroll
  for (int k = 0; k < kIt; k++) {
    const int i = tid + (int)blockDim.x * k;
    if (i < nw) {
      const int f = i / w4, j = i - f * w4;
      uint32_t* d = reinterpret_cast<uint32_t*>(T + f * Sp) + 4 * j;
      d[0] = r.x[k].x;
      d[1] = r.x[k].y;
      d[2] = r.x[k].z;
      d[3] = r.x[k].w;
    }
  }
  for (int i = tid + (int)blockDim.x * kIt; i < nw; i += blockDim.x) {  // (blocks under 256 threads)
    const int f = i / w4, j = i - f * w4;
    const uint4 y = reinterpret_cast<const uint4*>(E + (size_t)f * S)[j];
    uint32_t* d = reinterpret_cast<uint32_t*>(T + f * Sp) + 4 * j;
    d[0] = y.x;
    d[1] = y.y;
    d[2] = y.z;
    d[3] = y.w;
  }
  for (int k = tid; k < kMaxSlots + 64; k += blockDim.x) pk[k] = kAoEmpty;
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 2; u++) {
    const int s = tid + (int)blockDim.x * u;
    if (s < S && al[u] && (unsigned)(ds[u] - 1) < (unsigned)S) {
      const bool player = s < P;
      const bool immune = player && T[F_TIME_ALIVE * Sp + s] < p.spawn_immunity;
      const bool danger = T[F_NPC_TYPE * Sp + s] > 1;
      pk[ds[u] - 1] = ao_pack(s, T[F_ROW * Sp + s], T[F_COL * Sp + s], immune, danger, player);
    }
  }
  __syncthreads();
}
// listing tid's item word (a valid address whatever the mlist word: used only below the count)
__device__ __forceinline__ uint2 ao_listing_load(const ObsParams& p, int e, const AoStage& r) {
  const int own = min((r.mv >> 16) & 255, p.P - 1), slot = min((r.mv >> 24) & 15, kInv - 1);
  return p.items[((size_t)e * p.P + own) * kInv + slot];
}

// Workgroup -> (env, agent group) for a 1-D grid of n_envs * G workgroups. Workgroups are
// dispatched round-robin over the 8 XCDs (id % 8), each with its own L2: the G groups of an env
// go to one XCD back to back, so the env's staged columns come from HBM once and from that L2
// G - 1 times (with a 2-D grid an env's groups were n_envs workgroups apart: every group fetched
// them from HBM). Falls back to adjacent ids when n_envs % 8 != 0. Used by the wire kernel (same
// box: C5 at N = 1 375 -> 380 M) and the flat kernel (round 6: C4 308 -> 312 M same box, the
// kernel alone 1 % slower but the overlapped tick gets the HBM reads it no longer makes); the
// native kernel measured slower with it (round 6 again: C4-native 341 -> 339 M) and keeps the 2-D
// grid.
__device__ __forceinline__ void ao_env_group(int n_envs, int G, int& e, int& g) {
  const int id = blockIdx.x;
  if ((n_envs & 7) == 0) {
    const int x = id & 7, q = id >> 3;
    g = q % G;
    e = (q / G) * 8 + x;
  } else {
    e = id / G;
    g = id - e * G;
  }
}

// The window rows and item words of a workgroup's kAoAgents agents (g * kAoAgents ..), staged in
// LDS once per workgroup (every thread; one barrier inside): ws[(la * 15 + row) * 5 + k] = the 5
// aligned dwords holding window row `row` of agent la (its 15 materials start at byte
// (col - kVision) & 3 of them: 160 is a multiple of 4), is[la * kInv + k] = its item word k.
// The agent loops then issue no global load. On gfx9 vmcnt counts stores as well as loads and
// retires them in issue order, so a load prefetched inside the loop is waited on at the loop's
// back edge together with the stores issued after it -- as many of them as the compiler cannot
// prove were issued on every path (the variable zero runs): one agent's row stores drained before
// the next agent started.
constexpr int kAoWinRowBytes = 20;
constexpr int kAoWinAgentBytes = 15 * kAoWinRowBytes;  // 300
__host__ __device__ inline size_t ao_win_lds(int agents = kAoAgents) {
  return (size_t)agents * kAoWinAgentBytes + (size_t)agents * kInv * 8;
}
// positions of agents not in the realm are clamped so their (unused) window reads stay in the map
__device__ __forceinline__ int ao_clamp_pos(int x) { return min(max(x, kVision), kSize - 1 - kVision); }
// `before_barrier` runs after the LDS writes (every thread), ahead of the barrier that publishes them.
struct AoNoop {
  __device__ void operator()() const {}
};
template <int kAgents = kAoAgents, typename F = AoNoop>
__device__ inline void ao_stage_windows(const ObsParams& p, int e, int g, const int16_t* T, int Sp, uint32_t* ws, uint2* is,
                                        F before_barrier = F()) {
  const int tid = threadIdx.x, P = p.P;
  const int la = tid / 15, row = tid - 15 * la, a = g * kAgents + la;
  const bool win = tid < kAgents * 15 && a < P;
  uint32_t d[5] = {0u, 0u, 0u, 0u, 0u};
  if (win) {
    const int r = ao_clamp_pos(T[F_ROW * Sp + a]), c = ao_clamp_pos(T[F_COL * Sp + a]);
    const int base = (r - kVision + row) * kSize + c - kVision;
    const uint32_t* src = reinterpret_cast<const uint32_t*>(p.mat + (size_t)e * kTiles) + (base >> 2);
#pragma unroll
    for (int k = 0; k < 5; k++) d[k] = src[k];
  }
  uint2 iw = make_uint2(0u, 0u);
  const bool itm = tid < kAgents * kInv && g * kAgents + tid / kInv < P;
  if (itm) iw = p.items[((size_t)e * P + g * kAgents) * kInv + tid];
  if (win) {
#pragma unroll
    for (int k = 0; k < 5; k++) ws[tid * 5 + k] = d[k];  // tid = la * 15 + row
  }
  if (tid < kAgents * kInv) is[tid] = iw;
  before_barrier();
  __syncthreads();
}
// Per-lane byte offsets of window tiles t = lane + 64 i (i < 4) in an agent's staged rows
// (row(t) * 20 + col(t)), two 16-bit values per register
__device__ __forceinline__ void ao_win_offsets(int (&wo)[2]) {
  wo[0] = wo[1] = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int t = lane_id() + 64 * i;
    const int o = t < 225 ? (t / 15) * kAoWinRowBytes + t % 15 : 0;
    wo[i >> 1] |= o << (16 * (i & 1));
  }
}
__device__ __forceinline__ int ao_win_off(const int (&wo)[2], int i) { return (wo[i >> 1] >> (16 * (i & 1))) & 0xFFFF; }

// Entity.Query.window: ascending datastore rows within L-inf <= kVision; the first kNObs packed
// words go to visw. Returns the in-window count (uncapped).
__device__ __forceinline__ int ao_compact(const uint32_t (&pr)[kAoRows], int S, int r, int c, uint32_t* visw) {
  int nvis = 0;
  const uint32_t rc = (uint32_t)r | (uint32_t)c << 16;
#pragma unroll
  for (int i = 0; i < kAoRows; i++) {
    if (64 * i >= S) break;
    const uint32_t x = pr[i];
    const bool in = ao_in_window(x, rc);  // (an empty row is at (255, 255): outside)
    const uint64_t b = __ballot(in);
    const int pos = nvis + __popcll(b & lanes_below());
    if (in && pos < kNObs) visw[pos] = x;
    nvis += __popcll(b);
  }
  return nvis;
}

// Map offsets of the window tiles t = lane + 64 i (i < 4) from the agent's tile, two int16 per
// register (per-wave constants: an agent's 225 material loads are then one add each; the wire
// kernel's in-loop prefetch -- its few stores per record make the back-edge wait cheap, and the
// staging's LDS cost it a workgroup per CU: 0.089 -> 0.091 ms per 512 envs)
__device__ __forceinline__ void ao_window_offsets(int (&mo)[2]) {
  mo[0] = mo[1] = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int t = lane_id() + 64 * i;
    const int o = t < 225 ? (t / 15 - kVision) * kSize + t % 15 - kVision : 0;
    mo[i >> 1] |= (o & 0xFFFF) << (16 * (i & 1));
  }
}
__device__ __forceinline__ int ao_window_off(const int (&mo)[2], int i) {
  return (int)(int16_t)(uint16_t)((uint32_t)mo[i >> 1] >> (16 * (i & 1)));
}

// Passability of the 5 Move targets from the window materials (tile t in lane t & 63 of wm[t >> 6];
// the centre's 4 neighbours are all in wm[1])
__device__ __forceinline__ uint32_t ao_move_bits(uint32_t wm1) {
  uint32_t b = 0u;
#pragma unroll
  for (int d = 0; d < 5; d++) {
    const int t = (kVision + dir_dr(d)) * 15 + kVision + dir_dc(d);
    if (!impassable((int)__builtin_amdgcn_readlane((int)wm1, t - 64))) b |= 1u << d;
  }
  return b;
}

// Use.InventoryItem over the inventory (lane k holds slot k's item word; `have`: slot k occupied):
// common.h item_usable without its per-lane branches. Lane i < 8 reads skill level i (melee,
// range, mage, fishing, herbalism, prospecting, carving, alchemy: F_MELEE_LEVEL + 2 i), lane 8 the
// max of the combat levels; an item's requirement is the lane its type maps to (a 4-bit table,
// requirement_level's cases), fetched with one cross-lane read.
static_assert(F_ALCHEMY_LEVEL == F_MELEE_LEVEL + 14 && F_FISHING_LEVEL == F_MELEE_LEVEL + 6 &&
                  F_HERBALISM_LEVEL == F_MELEE_LEVEL + 8, "skill level fields");
__host__ __device__ constexpr uint64_t ao_req_lut() {  // type -> requirement lane (types 0..15)
  uint64_t m = 0;
  for (int t = 0; t < 16; t++) {
    const int k = (t >= T_SPEAR && t <= T_WAND) ? t - T_SPEAR : (t >= T_WHETSTONE && t <= T_RUNES) ? t - T_WHETSTONE
                  : (t >= T_ROD && t <= T_CHISEL) ? 3 + t - T_ROD : 8;
    m |= (uint64_t)k << (4 * t);
  }
  return m;
}
static_assert(T_RATION == 16 && T_POTION == 17, "requirement table: ration -> fishing, potion -> herbalism");
__device__ __forceinline__ uint64_t ao_usable_ballot(const int16_t* T, int Sp, int ti, uint2 it, bool have) {
  const int lane = ao_lane();
  int lv = 0;
  if (lane < 8) {
    lv = T[(F_MELEE_LEVEL + 2 * lane) * Sp + ti];
  } else if (lane == 8) {
    lv = max((int)T[F_MELEE_LEVEL * Sp + ti], max((int)T[F_RANGE_LEVEL * Sp + ti], (int)T[F_MAGE_LEVEL * Sp + ti]));
  }
  const int type = it_type(it);
  const int k = type < 16 ? (int)((ao_req_lut() >> (4 * type)) & 15u) : type == T_RATION ? 3 : type == T_POTION ? 4 : 8;
  const int req = __shfl(lv, k);
  const bool eq = type >= T_HAT && type <= T_RUNES && it_equipped(it);  // equip_slot(type) >= 0
  return __ballot(have && !it_price(it) && (eq || it_level(it) <= req));
}

// The 11 ActionTargets sections other than Buy.MarketItem as wave-uniform bit fields (SPEC §8,
// §9, §13 edits): bit k = entry k of the section.
struct AoSections {
  uint64_t s0, s1[2], s3, s4, s5[2], s6[2], s7[2], s8, s9, s10[2], s11;
};
struct AoAgent {
  int a, ti, r, c, gold, aid, nv, ninv, prev_price;  // ti: the agent's column index in T
  uint32_t mv;
};
template <bool kWrap>
__device__ __forceinline__ AoSections ao_sections(const ObsParams& p, const int16_t* T, int Sp, const uint32_t* visw,
                                                 const AoAgent& g, uint2 it) {
  const bool combat = (p.systems & NMMO_SYS_COMBAT) != 0;
  const bool item = (p.systems & NMMO_SYS_ITEM) != 0;
  const bool exch = item && (p.systems & NMMO_SYS_EXCHANGE) != 0;
  const bool no_give = kWrap && (p.wflags & kWrapObsNoGive);
  const bool no_danger = kWrap && (p.wflags & kWrapObsNoDangerous);
  const int lane = ao_lane();
  AoSections x;
  // over the visible rows: 1 AttackTarget, 5 GiveTarget, 7 GoldTarget (+ noop k = kNObs)
  x.s1[0] = x.s1[1] = x.s5[0] = x.s5[1] = x.s7[0] = x.s7[1] = 0ull;
#pragma unroll
  for (int h = 0; h < 2; h++) {
    if (64 * h >= g.nv) break;
    const int k = 64 * h + lane;
    bool tgt = false, st = false;
    if (k < g.nv) {
      const uint32_t w = visw[k];
      const int q = ao_slot(w);
      tgt = combat && q != g.a && linf(g.r, g.c, ao_row(w), ao_col(w)) <= 3 && !ao_immune(w) &&
            !(no_danger && ao_danger(w));
      st = ao_player(w) && q != g.a && ao_row(w) == g.r && ao_col(w) == g.c;
    }
    x.s1[h] = __ballot(tgt);
    const uint64_t sb = __ballot(st);
    if (item && !no_give) x.s5[h] = sb;
    if (exch && !no_give) x.s7[h] = sb;
  }
  x.s1[1] |= 1ull << (kNObs - 64);
  x.s5[1] |= 1ull << (kNObs - 64);
  x.s7[1] |= 1ull << (kNObs - 64);
  // over the inventory (lane k holds slot k's item word): 3 Destroy, 4 GiveItem, 9 SellItem,
  // 11 Use (+ noop k = kInv)
  const bool have = lane < g.ninv;
  const bool fr = have && !it_equipped(it) && !it_price(it);
  const uint64_t bfr = __ballot(fr);
  x.s3 = (item ? bfr : 0ull) | 1ull << kInv;
  x.s4 = (item && !no_give ? bfr : 0ull) | 1ull << kInv;
  x.s9 = (exch ? __ballot(have && !it_equipped(it)) : 0ull) | 1ull << kInv;
  x.s11 = (item ? ao_usable_ballot(T, Sp, g.ti, it, have) : 0ull) | 1ull << kInv;
  // closed forms: 0 Style, 6 GoldPrice (k < gold), 8 Move, 10 SellPrice (all but the wrapper's
  // last price)
  x.s0 = combat ? low_bits(kSecN[0]) : 0ull;
  x.s6[0] = x.s6[1] = x.s10[0] = x.s10[1] = 0ull;
  if (exch) {
    const int ng = no_give ? min(g.gold, 1) : min(g.gold, kSecN[6]);
    x.s6[0] = low_bits(ng);
    x.s6[1] = low_bits(ng - 64);
    x.s10[0] = low_bits(kSecN[10]);
    x.s10[1] = low_bits(kSecN[10] - 64);
    if constexpr (kWrap) {
      const int pp = g.prev_price;
      if ((p.wflags & kWrapObsPrice) && pp >= 0 && pp < kSecN[10]) {
        // (no runtime index into x: one put the whole struct in scratch, whose loads then waited
        // for every store the kernel had issued)
        const uint64_t clr = ~(1ull << (pp & 63));
        if (pp < 64) x.s10[0] &= clr;
        else x.s10[1] &= clr;
      }
    }
  }
  x.s8 = g.mv;
  return x;
}

// The sections into a bit image: kFlat = flat entry order (1,586 bits, Buy.MarketItem left 0),
// else the wire order (561 bits)
template <bool kFlat, int kW>
__device__ __forceinline__ void ao_image(const AoSections& x, uint32_t (&img)[kW]) {
#pragma unroll
  for (int d = 0; d < kW; d++) img[d] = 0u;
#define AO_PUT(k, lo, hi) put_field<kFlat ? sec_flat(k) : sec_wire(k), kSecN[k], kW>(img, lo, hi)
  AO_PUT(0, x.s0, 0ull);
  AO_PUT(1, x.s1[0], x.s1[1]);
  AO_PUT(3, x.s3, 0ull);
  AO_PUT(4, x.s4, 0ull);
  AO_PUT(5, x.s5[0], x.s5[1]);
  AO_PUT(6, x.s6[0], x.s6[1]);
  AO_PUT(7, x.s7[0], x.s7[1]);
  AO_PUT(8, x.s8, 0ull);
  AO_PUT(9, x.s9, 0ull);
  AO_PUT(10, x.s10[0], x.s10[1]);
  AO_PUT(11, x.s11, 0ull);
#undef AO_PUT
}

}  // namespace nmmo
