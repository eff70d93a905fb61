// common.h — device-side constants and primitives of the gfx950 stepper (SPEC.md §1-§3).
// Product code: the oracle under oracle/ restates these independently (it shares nothing but
// include/nmmo_hip.h), so a wrong constant here shows up as a parity failure.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/nmmo_hip.h"

namespace nmmo {

constexpr int kSize = NMMO_MAP_SIZE;  // 160
constexpr int kTiles = NMMO_MAP_TILES;
constexpr int kLo = 16, kHi = 143, kCenter = 128, kVision = 7, kNObs = 100;
constexpr int kBitmapWords = kTiles / 32;  // 800 depleted-tile bitmap words per env
constexpr int kNFLive = F_DROP_TOOL + 1;   // entity fields carried through LDS (45)
constexpr int kMaxSlots = 384;
constexpr int kHeads = NMMO_N_ACTION_HEADS;

enum Material : int {
  M_VOID, M_WATER, M_GRASS, M_SCRUB, M_FOILAGE, M_STONE, M_SLAG, M_ORE, M_STUMP, M_TREE,
  M_FRAGMENT, M_CRYSTAL, M_WEEDS, M_HERB, M_OCEAN, M_FISH
};
enum Purpose : uint32_t {
  P_MAPSEL = 1, P_SPAWN_OFFSET = 2, P_RESILIENT = 3, P_NPC_SPAWN = 4, P_NPC_MOVE = 5,
  P_RESPAWN = 6, P_BUY_ORDER = 7, P_TASK = 8
};

// ---------------------------------------------------------------- items (SPEC §9)
constexpr int kInv = NMMO_INV_SLOTS;
enum ItemType : int {
  T_HAT = 2, T_TOP, T_BOTTOM, T_SPEAR, T_BOW, T_WAND, T_ROD, T_GLOVES, T_PICKAXE, T_AXE, T_CHISEL,
  T_WHETSTONE, T_ARROW, T_RUNES, T_RATION, T_POTION
};
// item = uint2: x = type | level<<5 | equipped<<9 | listed_price<<10 | listed_tick<<17,
//               y = quantity | row<<16 ; type 0 = empty slot
__host__ __device__ inline int it_type(uint2 w) { return (int)(w.x & 31u); }
__host__ __device__ inline int it_level(uint2 w) { return (int)((w.x >> 5) & 15u); }
__host__ __device__ inline int it_equipped(uint2 w) { return (int)((w.x >> 9) & 1u); }
__host__ __device__ inline int it_price(uint2 w) { return (int)((w.x >> 10) & 127u); }
__host__ __device__ inline int it_ltick(uint2 w) { return (int)((w.x >> 17) & 2047u); }
__host__ __device__ inline int it_qty(uint2 w) { return (int)(w.y & 0xFFFFu); }
__host__ __device__ inline int it_row(uint2 w) { return (int)(w.y >> 16); }
__host__ __device__ inline int item_attack(int type, int level, int style) {
  return (type == T_SPEAR + style || type == T_WHETSTONE + style) ? 5 + 5 * level : 0;
}
__host__ __device__ inline int item_defense(int type, int level) {
  return (type >= T_HAT && type <= T_BOTTOM) ? 3 * level : (type >= T_ROD && type <= T_CHISEL) ? 2 * level : 0;
}
// level an item requires of its user; T is field-major with stride S (SPEC §9)
__device__ inline int requirement_level(const int16_t* T, int S, int p, int type) {
  if (type >= T_SPEAR && type <= T_WAND) return T[(F_MELEE_LEVEL + 2 * (type - T_SPEAR)) * S + p];
  if (type >= T_WHETSTONE && type <= T_RUNES) return T[(F_MELEE_LEVEL + 2 * (type - T_WHETSTONE)) * S + p];
  if (type >= T_ROD && type <= T_CHISEL) return T[(F_FISHING_LEVEL + 2 * (type - T_ROD)) * S + p];
  if (type == T_RATION) return T[F_FISHING_LEVEL * S + p];
  if (type == T_POTION) return T[F_HERBALISM_LEVEL * S + p];
  return max((int)T[F_MELEE_LEVEL * S + p], max((int)T[F_RANGE_LEVEL * S + p], (int)T[F_MAGE_LEVEL * S + p]));
}
__host__ __device__ inline int equip_slot(int type) {  // hat top bottom held ammo; -1 consumable
  return (type >= T_HAT && type <= T_BOTTOM) ? type - T_HAT
         : (type >= T_SPEAR && type <= T_CHISEL) ? 3
         : (type >= T_WHETSTONE && type <= T_RUNES) ? 4 : -1;
}

// bit m set <=> material m is impassable (Void, Water, Stone, Ocean, Fish)
constexpr uint32_t kImpassableMask = (1u << M_VOID) | (1u << M_WATER) | (1u << M_STONE) |
                                     (1u << M_OCEAN) | (1u << M_FISH);
__host__ __device__ inline bool impassable(int m) { return (kImpassableMask >> m) & 1u; }

__host__ __device__ inline uint32_t respawn_u32(int base) {
  switch (base) {
    case M_FOILAGE: return 107374182u;
    case M_TREE: case M_ORE: case M_CRYSTAL: return 429496729u;
    case M_HERB: case M_FISH: return 85899345u;
    default: return 0u;
  }
}

__host__ __device__ inline int level_at_exp(int exp) {
  const int thr[10] = {0, 90, 250, 500, 900, 1500, 2400, 3700, 5500, 8000};
  int l = 0;
#pragma unroll
  for (int i = 0; i < 10; i++) l += exp >= thr[i];
  return l;
}
// (a select chain: a runtime index into a constant array is a global load on the device, and in
// the tick it came after the phase's stores -- vmcnt retires in order -- so it drained them)
__host__ __device__ inline int exp_at_level(int level) {
  return level <= 1 ? 0 : level == 2 ? 90 : level == 3 ? 250 : level == 4 ? 500 : level == 5 ? 900
       : level == 6 ? 1500 : level == 7 ? 2400 : level == 8 ? 3700 : level == 9 ? 5500 : 8000;
}

__host__ __device__ inline int dir_dr(int d) { return d == 0 ? -1 : d == 1 ? 1 : 0; }
__host__ __device__ inline int dir_dc(int d) { return d == 2 ? 1 : d == 3 ? -1 : 0; }

__host__ __device__ inline int iabs(int x) { return x < 0 ? -x : x; }
__host__ __device__ inline int linf(int r0, int c0, int r1, int c1) {
  int a = iabs(r0 - r1), b = iabs(c0 - c1);
  return a > b ? a : b;
}

// ---------------------------------------------------------------- RNG (SPEC §2)
__host__ __device__ inline uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

struct U4 { uint32_t x, y, z, w; };

__host__ __device__ inline U4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                     uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; r++) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return U4{c0, c1, c2, c3};
}
__host__ __device__ inline U4 draw(uint64_t seed, uint32_t tick, uint32_t purpose,
                                   uint32_t index, uint32_t sub) {
  return philox(tick, purpose, index, sub, (uint32_t)seed, (uint32_t)(seed >> 32));
}
__host__ __device__ inline uint32_t uniform_n(uint32_t u, uint32_t n) {
  return (uint32_t)(((uint64_t)u * n) >> 32);
}

// ---------------------------------------------------------------- map hash (SPEC §3)
__host__ __device__ inline uint32_t h32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

// ---------------------------------------------------------------- LDS/wave helpers
__device__ inline int lane_id() { return threadIdx.x & 63; }
__device__ inline int wave_id() { return threadIdx.x >> 6; }
__device__ inline uint64_t lanes_below() { return (1ull << lane_id()) - 1ull; }

// Inclusive prefix sum over the 64 lanes of a wave in six DPP moves: row_shr 1/2/4/8 scan each
// 16-lane row, then row_bcast:15 and row_bcast:31 carry row totals into the rows above
// (disabled rows and out-of-row sources read the `old` operand, 0).
__device__ __forceinline__ int wave_incl_scan(int x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, false);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, false);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, false);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, false);  // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
  return x;
}
__host__ __device__ __forceinline__ uint32_t i16pack(int lo, int hi) {
  return (uint32_t)(uint16_t)(int16_t)lo | ((uint32_t)(uint16_t)(int16_t)hi << 16);
}
// Sum over the 64 lanes of a wave (all lanes active), wave-uniform.
__device__ __forceinline__ int wave_sum(int x) { return __builtin_amdgcn_readlane(wave_incl_scan(x), 63); }

// zero [lo, hi) of a float row with 16-byte stores on the aligned body (wave-cooperative)
__device__ inline void wave_zero(float* row, int lo, int hi) {
  const int lane = lane_id();
  const uintptr_t a = reinterpret_cast<uintptr_t>(row + lo);
  int head = (int)(((16 - (a & 15)) & 15) >> 2);
  if (head > hi - lo) head = hi - lo;
  if (lane < head) row[lo + lane] = 0.f;
  const int body = (hi - lo - head) >> 2;
  float4* p4 = reinterpret_cast<float4*>(row + lo + head);
  for (int i = lane; i < body; i += 64) p4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  const int tail0 = lo + head + body * 4;
  if (tail0 + lane < hi) row[tail0 + lane] = 0.f;
}
__device__ inline bool item_usable(const int16_t* T, int S, int p, uint2 w) {
  if (it_price(w)) return false;
  if (equip_slot(it_type(w)) >= 0 && it_equipped(w)) return true;
  return it_level(w) <= requirement_level(T, S, p, it_type(w));
}
// column col of an Inventory / Market obs row (nmmo ItemState order, SPEC §9)
__device__ inline float item_col(uint2 w, int owner_id, int col) {
  const int type = it_type(w), lvl = it_level(w);
  switch (col) {
    case 0: return (float)it_row(w);
    case 1: return (float)type;
    case 2: return (float)owner_id;
    case 3: return (float)lvl;
    case 4: return 0.f;
    case 5: return (float)it_qty(w);
    case 6: case 7: case 8: return (float)item_attack(type, lvl, col - 6);
    case 9: case 10: case 11: return (float)item_defense(type, lvl);
    case 12: return type == T_POTION ? (float)(50 + 5 * lvl) : 0.f;
    case 13: return type == T_RATION ? (float)(50 + 5 * lvl) : 0.f;
    case 14: return (float)it_equipped(w);
    default: return (float)it_price(w);
  }
}
// inventory of one player: kInv slots, occupied prefix in ascending row order
__device__ inline int inv_count(const uint2* inv) {
  int n = 0;
  while (n < kInv && it_type(inv[n])) n++;
  return n;
}
__device__ inline int inv_find(const uint2* inv, int row) {
  for (int k = 0; k < kInv; k++) {
    const uint2 w = inv[k];
    if (!it_type(w)) break;
    if (it_row(w) == row) return k;
  }
  return -1;
}
__device__ inline void inv_remove(uint2* inv, int k) {
  for (int j = k; j < kInv - 1; j++) inv[j] = inv[j + 1];
  inv[kInv - 1] = make_uint2(0u, 0u);
}
__device__ inline void inv_insert(uint2* inv, uint2 w) {  // caller checked room
  int k = inv_count(inv);
  while (k > 0 && it_row(inv[k - 1]) > it_row(w)) {
    inv[k] = inv[k - 1];
    k--;
  }
  inv[k] = w;
}
__device__ inline int inv_stack(const uint2* inv, int type, int level) {  // ammunition stacks
  if (type < T_WHETSTONE || type > T_RUNES) return -1;
  for (int k = 0; k < kInv; k++) {
    const uint2 w = inv[k];
    if (!it_type(w)) break;
    if (it_type(w) == type && it_level(w) == level) return k;
  }
  return -1;
}

// lane `lane` of `old` <- the wave-uniform `val`: v_cmp + v_cndmask. (An inline-asm
// v_writelane_b32 with the lane select in M0 is one op cheaper but mis-set ~1 in 10^3 masks on
// gfx950 — a hazard the compiler's recognizer cannot see inside asm — so it is not used.)
__device__ inline uint32_t writelane_u32(uint32_t old, uint32_t val, uint32_t lane) {
  return lane_id() == (int)lane ? val : old;
}

// The wave totals below wave w and of all nw waves, read from an 8-entry buffer in one fixed
// pass (all 8 entries are read, those of waves >= nw masked): a loop to the runtime wave count
// compiles to a general unrolled loop with remainder handling, ~100 instructions per prefix.
__device__ __forceinline__ int wave_tot_below(const int* wave_tot, int w, int nw, int* total) {
  int base = 0, sum = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int ti = wave_tot[i];
    const int t = i < nw ? ti : 0;
    base += i < w ? t : 0;
    sum += t;
  }
  *total = sum;
  return base;
}

// Block-wide exclusive prefix sum of an int in thread order (<= 8 waves); *total gets the sum.
// One barrier: `wave_tot` (>= 8 ints of LDS) must not be the buffer of the previous call (it
// may still be read), so consecutive calls alternate two buffers. All accesses before the call
// are ordered before all accesses after it by that barrier.
__device__ inline int block_prefix_sum(int v, int* wave_tot, int* total) {
  const int w = __builtin_amdgcn_readfirstlane(wave_id()), nw = (blockDim.x + 63) >> 6;
  const int x = wave_incl_scan(v);
  if (lane_id() == 63) wave_tot[w] = x;
  __syncthreads();
  return wave_tot_below(wave_tot, w, nw, total) + x - v;
}

// Block-wide exclusive prefix count of a 0/1 predicate in thread order (<= 8 waves); same
// buffer rule as block_prefix_sum. Returns the exclusive count; *total gets the sum.
__device__ inline int block_prefix_count(bool pred, int* wave_tot, int* total) {
  const uint64_t b = __ballot(pred);
  const int w = __builtin_amdgcn_readfirstlane(wave_id()), nw = (blockDim.x + 63) >> 6;
  if (lane_id() == 0) wave_tot[w] = __popcll(b);
  __syncthreads();
  return wave_tot_below(wave_tot, w, nw, total) + __popcll(b & lanes_below());
}

// ---------------------------------------------------------------- visibility grid
// Visibility grid: 16x16-tile cells; a 15x15 window touches at most kWinRows x kWinRows
// cells. Players and NPCs are bucketed separately: grid cell ids [0, kCells) hold players,
// [kCells, 2 kCells) NPCs, so the cells c0..c1 of one grid row are one contiguous range in
// either half.
constexpr int kCellShift = 4;
constexpr int kGrid = (kSize + (1 << kCellShift) - 1) >> kCellShift;  // 10
constexpr int kCells = kGrid * kGrid;
constexpr int kGridCells = 2 * kCells;
constexpr int kWinRows = (14 + (1 << kCellShift) - 1) / (1 << kCellShift) + 1;  // 2
__host__ __device__ constexpr size_t grid_lds_bytes(int S) {  // gstart | glist
  return (((size_t)(kGridCells + 1) * 4 + 15) & ~(size_t)15) + (((size_t)S * 4 + 15) & ~(size_t)15);
}
// first / last grid row and first / last grid column of the window around (r, c)
__device__ __forceinline__ int4 grid_window(int r, int c) {
  return make_int4(max(r - 7, 0) >> kCellShift, min(r + 7, kSize - 1) >> kCellShift,
                   max(c - 7, 0) >> kCellShift, min(c + 7, kSize - 1) >> kCellShift);
}

// Counting sort of the block's entities into the grid. Every thread calls it (it holds
// barriers) with its entity's grid cell id (or -1) and payload; blockDim.x >= 64. On return
// gstart[cell] .. gstart[cell + 1] index cell's payloads in glist.
__device__ __forceinline__ void grid_build(int* gstart, uint32_t* glist, int cell, uint32_t entry) {
  const int tid = threadIdx.x, nt = blockDim.x;
  for (int k = tid; k <= kGridCells; k += nt) gstart[k] = 0;
  __syncthreads();
  const int gi = cell >= 0 ? atomicAdd(&gstart[cell], 1) : 0;
  __syncthreads();
  if (tid < 64) {  // wave 0: in-place exclusive scan, kPer consecutive cells per lane
    constexpr int kPer = (kGridCells + 63) / 64;
    const int b = tid * kPer;
    int loc[kPer], sum = 0;
#pragma unroll
    for (int j = 0; j < kPer; j++) {
      loc[j] = b + j < kGridCells ? gstart[b + j] : 0;
      sum += loc[j];
    }
    const int x = wave_incl_scan(sum);
    int ex = x - sum;
#pragma unroll
    for (int j = 0; j < kPer; j++) {
      if (b + j < kGridCells) gstart[b + j] = ex;
      ex += loc[j];
    }
    if (tid == 63) gstart[kGridCells] = x;
  }
  __syncthreads();
  if (cell >= 0) glist[gstart[cell] + gi] = entry;
  __syncthreads();
}

// Visit the grid entries glist[i0, i1) (bits 0-7 column, 8-15 row) within L-inf 7 of (r, c):
// f(entry, L-inf distance, index). Loads are issued four at a time ahead of their uses.
template <class Fn>
__device__ __forceinline__ void grid_scan(const uint32_t* __restrict__ glist, int i0, int i1, int r,
                                          int c, Fn&& f) {
  auto one = [&](uint32_t v, int i) {
    const int d = max(abs((int)((v >> 8) & 255) - r), abs((int)(v & 255) - c));
    if (d <= 7) f(v, d, i);
  };
  int i = i0;
  for (; i + 4 <= i1; i += 4) {
    const uint32_t v0 = glist[i], v1 = glist[i + 1], v2 = glist[i + 2], v3 = glist[i + 3];
    one(v0, i);
    one(v1, i + 1);
    one(v2, i + 2);
    one(v3, i + 3);
  }
  for (; i < i1; i++) one(glist[i], i);
}

// ---------------------------------------------------------------- packed-row scans
// rp: per datastore row r | c<<8 | slot<<16 (| flags<<25), -1 = no entity; padded with -1 to a
// multiple of 4 entries and 16-B aligned so a scan reads 4 rows per ds_read_b128, branch-free.
__host__ __device__ inline int rp_groups(int S) { return (S + 4) >> 2; }

// slot of the k-th (0-based) entity within L-inf <= kVision of (r, c) in row order, or -1
__device__ inline int kth_visible(const int* __restrict__ rp, int S, int r, int c, int k) {
  const int4* rp4 = reinterpret_cast<const int4*>(rp);
  const int ng = rp_groups(S);
  int cnt = 0, tgt = -1;
  for (int g = 0; g < ng; g++) {
    const int4 q = rp4[g];
    const int vv[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int v = vv[j];
      const bool vis = v >= 0 && linf(r, c, v & 255, (v >> 8) & 255) <= kVision;
      tgt = (vis && cnt == k) ? ((v >> 16) & 511) : tgt;
      cnt += vis;
    }
    if (cnt > k) break;
  }
  return tgt;
}

}  // namespace nmmo
