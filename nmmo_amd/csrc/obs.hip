// obs.hip — per-agent observation gather (SPEC.md §8) and the scripted masked-uniform policy
// (SPEC.md §10).
//
// Replaces Env._compute_observations + pufferlib's flatten/pad (the buffer the reference
// receives from pool.recv(), clean_pufferl.py:293, and decodes with unpack_batched_obs,
// baseline_policy.py:41). Output: float32 [n_envs][P][23,987] in pufferlib sorted-key order.
//
// Roofline: this kernel is HBM-write-bound — 95,948 B written per agent row against ~0.3 KB of
// reads (the env's entity columns are staged once per workgroup in LDS and shared by its 16
// agents; the 225 map bytes and the 8-KB Task embedding per agent come from L2). One wave owns
// one agent row at a time: it compacts the agent's visible entities with a ballot/prefix-popcount
// over datastore rows (the nmmo window order) into LDS, then streams the row with coalesced
// stores — 16-byte stores for the zero runs (unseen Entity rows, Market), dword stores elsewhere.
// Every global load of the next agent is issued ahead of the current row's bulk stores, so the
// store stream never waits on a load (vmcnt retires in issue order).
#include "kernels.h"

namespace nmmo {

constexpr int kObsAgentsPerBlock = 16;  // expand_kernel's shape
constexpr int kObsWaves = 4;
#ifndef NMMO_OBS_FLAT_APB  // (A/B knob: tools/debug/variants.py)
#define NMMO_OBS_FLAT_APB 16
#endif
// obs_kernel: agents per workgroup, 4 per wave; the env's staged columns are shared by them
constexpr int kFlatAgents = NMMO_OBS_FLAT_APB, kFlatWaves = kFlatAgents / 4;
constexpr int kObsFields = F_DS_ROW + 1;  // 0..30 obs columns, alive, ds_row
// LDS: entity fields | row->slot | per-wave visible list | per-wave inventory | market listings
// (item words, 8 B, then price | owner << 8, 2 B) | per-wave 15x15 window materials.
// (The native and wire layouts have their own kernels: native_obs.hip, wire_obs.hip.)
__host__ __device__ inline size_t obs_lds_bytes(int S) {
  return (((size_t)kObsFields * S * 2 + 15) & ~(size_t)15) + (((size_t)(S + 1) * 4 + 15) & ~(size_t)15) +
         (size_t)kFlatWaves * 128 * 2 + (size_t)kFlatWaves * kInv * 8 + (size_t)kFlatWaves * 256 +
         (size_t)NMMO_MARKET_ROWS * 10;
}

// Plain (temporal) stores. Measured on MI355X (same-box A/B): __builtin_nontemporal_store
// ("nt") made the C4 obs kernel 33% slower (3.52 vs 2.65 ms per launch); building every row
// from 16-byte stores (4 consecutive elements per lane) was 54% slower (3.25 vs 2.11 ms: the
// per-element section dispatch doubled the VGPRs and halved occupancy).
__device__ __forceinline__ void obs_st(float* p, float v) { *p = v; }

__device__ __forceinline__ void obs_st4(float4* p, float4 v) { *p = v; }

// zero bytes [lo, hi) of a row (lo, hi even): int16 stores up to 16-B alignment, then 16-B stores
__device__ inline void wave_zero_bytes(uint8_t* row, int lo, int hi) {
  const int lane = lane_id();
  const uintptr_t a = reinterpret_cast<uintptr_t>(row + lo);
  int head = (int)((16 - (a & 15)) & 15);
  if (head > hi - lo) head = hi - lo;
  if (2 * lane < head) reinterpret_cast<int16_t*>(row + lo)[lane] = 0;
  const int body = (hi - lo - head) >> 4;
  uint4* p4 = reinterpret_cast<uint4*>(row + lo + head);
  for (int i = lane; i < body; i += 64) p4[i] = make_uint4(0u, 0u, 0u, 0u);
  const int t0 = lo + head + body * 16;
  if (t0 + 2 * lane < hi) reinterpret_cast<int16_t*>(row + t0)[lane] = 0;
}

// native layout (SPEC §8b): int16 part offsets, env stride, two int16 per dword store
constexpr int kNatEntity = 2, kNatInv = kNatEntity + kNObs * NMMO_N_ENTITY_COLS,
              kNatTile = kNatInv + kInv * 16, kNatTask = kNatTile + 225 * 3;
static_assert(kNatTask < NMMO_NATIVE_I16, "native int16 part overflows its row");
__host__ __device__ inline size_t native_env_bytes(int P) {
  return (size_t)P * NMMO_NATIVE_ROW_BYTES + NMMO_NATIVE_MARKET_BYTES;
}

// One agent's view for the ActionTargets sections (SPEC §8, §9, §13 edits).
struct MaskCtx {
  int a, r, c, nv, gold, ninv, prev_price;
  uint32_t movebits;  // bit d: the tile in direction d is passable
  bool combat, item, exch, no_give;
};

// The 12 ActionTargets sections in flat order: [lo, lo + n) of the mask part of the row.
__device__ __forceinline__ void mask_section(const ObsParams& p, int sec, int& lo, int& n) {
  switch (sec) {
    case 0: lo = p.o_style; n = p.o_target - p.o_style; break;
    case 1: lo = p.o_target; n = kNObs + 1; break;
    case 2: lo = p.o_buy; n = NMMO_MARKET_ROWS + 1; break;
    case 3: lo = p.o_destroy; n = kInv + 1; break;
    case 4: lo = p.o_give_item; n = kInv + 1; break;
    case 5: lo = p.o_give_target; n = kNObs + 1; break;
    case 6: lo = p.o_gg_price; n = p.o_gg_target - p.o_gg_price; break;
    case 7: lo = p.o_gg_target; n = kNObs + 1; break;
    case 8: lo = p.o_move; n = p.o_sell_item - p.o_move; break;
    case 9: lo = p.o_sell_item; n = kInv + 1; break;
    case 10: lo = p.o_sell_price; n = p.o_use - p.o_sell_price; break;
    default: lo = p.o_use; n = p.o_agent_id - p.o_use; break;
  }
}

// Entry k of section sec (the section id is wave-uniform: no lane evaluates another section's
// predicate). Buy.MarketItem reads the packed listings (price | owner << 8) in either layout.
template <bool kWrap>
__device__ __forceinline__ bool mask_value(const ObsParams& p, const int16_t* T, int S,
                                           const int16_t* vis, const uint2* inv, const uint16_t* mpo,
                                           int nm, const MaskCtx& m, int sec, int k) {
  auto free_item = [&](int q) { return q < m.ninv && !it_equipped(inv[q]) && !it_price(inv[q]); };
  auto same_tile = [&](int q) {
    const int s = vis[q];
    return s < p.P && s != m.a && T[F_ROW * S + s] == m.r && T[F_COL * S + s] == m.c;
  };
  bool v;
  switch (sec) {
    case 0: v = m.combat; break;
    case 1:
      if (k == kNObs) {
        v = true;
      } else if (!m.combat || k >= m.nv) {
        v = false;
      } else {
        const int q = vis[k];
        v = q != m.a && linf(m.r, m.c, T[F_ROW * S + q], T[F_COL * S + q]) <= 3 &&
            !(q < p.P && T[F_TIME_ALIVE * S + q] < p.spawn_immunity);
        if constexpr (kWrap)
          if ((p.wflags & kWrapObsNoDangerous) && T[F_NPC_TYPE * S + q] > 1) v = false;
      }
      break;
    case 2:
      v = k == NMMO_MARKET_ROWS ||
          (m.exch && k < nm && (int)(mpo[k] & 255u) <= m.gold && (int)(mpo[k] >> 8) != m.a);
      break;
    case 3: v = k == kInv || (m.item && free_item(k)); break;
    case 4: v = k == kInv || (!m.no_give && m.item && free_item(k)); break;
    case 5: v = k == kNObs || (!m.no_give && m.item && k < m.nv && same_tile(k)); break;
    case 6: v = m.exch && k < m.gold && (!m.no_give || k == 0); break;
    case 7: v = k == kNObs || (!m.no_give && m.exch && k < m.nv && same_tile(k)); break;
    case 8: v = (m.movebits >> k) & 1u; break;
    case 9: v = k == kInv || (m.exch && k < m.ninv && !it_equipped(inv[k])); break;
    case 10:
      v = m.exch;
      if constexpr (kWrap)
        if ((p.wflags & kWrapObsPrice) && k == m.prev_price) v = false;
      break;
    default: v = k == kInv || (m.item && k < m.ninv && item_usable(T, S, m.a, inv[k])); break;
  }
  return v;
}

// Section kSec of the ActionTargets as float32 0/1 straight into a flat row: the section is a
// template constant, so mask_section / mask_value fold to straight-line code (the generic
// (section, chunk) loop spent ~1.3k scalar and branch instructions per agent on the dispatch).
template <int kSec, bool kWrap>
__device__ __forceinline__ void mask_sec_f32(const ObsParams& p, const int16_t* T, int S, const int16_t* vis,
                                             const uint2* inv, const uint16_t* mpo, int nm, const MaskCtx& m,
                                             float* row) {
  int lo, n;
  mask_section(p, kSec, lo, n);
  for (int k = lane_id(); k < n; k += 64)
    obs_st(&row[lo + k], mask_value<kWrap>(p, T, S, vis, inv, mpo, nm, m, kSec, k) ? 1.f : 0.f);
}

// Passability of the 5 move targets from the prefetched window materials: tile t of the 15x15
// window sits in lane t & 63 of register t >> 6; the centre's 4 neighbours (t = 97, 111, 112,
// 113, 127) are all in register 1.
__device__ __forceinline__ uint32_t move_bits(uint32_t wm1) {
  uint32_t b = 0u;
#pragma unroll
  for (int d = 0; d < 5; d++) {
    const int t = (kVision + dir_dr(d)) * 15 + kVision + dir_dc(d);
    if (!impassable((int)__builtin_amdgcn_readlane((int)wm1, t - 64))) b |= 1u << d;
  }
  return b;
}

// Flat rows: each agent's global loads (its 12 item words, 15x15 window materials, Task
// embedding) are issued before the previous agent's remaining ~130 stores (vmcnt retires in
// issue order, so a load issued after a store stream waits for all of it; issued ahead of >= 63
// younger stores it costs no wait at all).
#ifndef NMMO_OBS_TASK_REGS  // (A/B knobs: tools/debug/variants.py)
#define NMMO_OBS_TASK_REGS 0  // (32 before the Task section was kept across steps: 156 VGPRs)
#endif
// Task embedding dwords per lane held in registers (2,048 per row): the incremental variant writes
// a Task section once per episode and reads it in place; the full-write variant (every row every
// launch: an unbound or untracked buffer, NMMO_OBS_REZERO) prefetches its first 2,048 floats with
// the agent's other loads, so its Task stores never wait behind the Tile stores issued before them.
#ifndef NMMO_OBS_FULL_TREGS  // (A/B knobs: 0 and 4 = the round-4 full write)
#define NMMO_OBS_FULL_TREGS 32
#endif
#ifndef NMMO_OBS_FULL_WPE
#define NMMO_OBS_FULL_WPE 3
#endif
constexpr int kTaskRegsFull = NMMO_OBS_FULL_TREGS;

// kWrap: the wrapper's observation() edits are compiled in (SPEC §13). kFull: no row state (every
// row written in full, Task from registers); 3 waves per SIMD (the registers take it past 128).
#ifndef NMMO_OBS_WPE  // 4 waves per SIMD: the wrapper variant would take 129 VGPRs (3 waves) and
#define NMMO_OBS_WPE 4  // fits 128 with a 20-B spill instead; the plain one is 128 either way
#endif
template <bool kWrap, bool kFull>
__global__ void __launch_bounds__(64 * kFlatWaves)
__attribute__((amdgpu_waves_per_eu(kFull ? NMMO_OBS_FULL_WPE : NMMO_OBS_WPE, kFull ? NMMO_OBS_FULL_WPE : NMMO_OBS_WPE)))
obs_kernel(ObsParams p) {
  constexpr int kTaskRegs = kFull ? kTaskRegsFull : NMMO_OBS_TASK_REGS;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int S = p.S;
  int16_t* T = reinterpret_cast<int16_t*>(smem);
  // datastore row k -> slot | row << 16 | col << 24 of the entity on it (0xFFFFFFFF: none)
  uint32_t* rowpk = reinterpret_cast<uint32_t*>(smem + (((size_t)kObsFields * S * 2 + 15) & ~(size_t)15));
  int16_t* vis_all = reinterpret_cast<int16_t*>(rowpk + ((((size_t)(S + 1) * 4 + 15) & ~(size_t)15) / 4));
  uint2* inv_all = reinterpret_cast<uint2*>(vis_all + kFlatWaves * 128);
  uint2* mitem = inv_all + kFlatWaves * kInv;  // listed item words
  uint16_t* mpo = reinterpret_cast<uint16_t*>(mitem + NMMO_MARKET_ROWS);  // price | owner << 8
  uint8_t* wmat_all = reinterpret_cast<uint8_t*>(mpo + NMMO_MARKET_ROWS);  // per-wave 15x15 materials
#ifdef NMMO_OBS_XCD  // A/B knob: 1-D grid, an env's groups on one XCD (as agent_obs.h ao_env_group)
  const int G = (p.P + kFlatAgents - 1) / kFlatAgents, ne = p.env_list ? p.n_list : p.n_envs;
  int el, g;
  if ((ne & 7) == 0) {
    const int x = blockIdx.x & 7, q = blockIdx.x >> 3;
    g = q % G;
    el = (q / G) * 8 + x;
  } else {
    el = blockIdx.x / G;
    g = blockIdx.x - el * G;
  }
  const int e = p.env_list ? p.env_list[el] : el;
#else
  const int e = p.env_list ? p.env_list[blockIdx.x] : (int)blockIdx.x, g = blockIdx.y;
#endif
  if ((unsigned)e >= (unsigned)p.n_envs) return;  // a bad list id (the tick records it)
  const int tid = threadIdx.x;
  const int nm = p.mcount[e];
  for (int j = tid; j < nm; j += blockDim.x) {  // end-of-tick listings, ascending row
    const int v = p.mlist[(size_t)e * NMMO_MARKET_ROWS + j];
    const int own = (v >> 16) & 255, slot = (v >> 24) & 15;
    const uint2 wd = p.items[((size_t)e * p.P + own) * kInv + slot];
    mpo[j] = (uint16_t)(it_price(wd) | own << 8);
    mitem[j] = wd;
  }
  {
    const int16_t* src = p.ent + (size_t)e * NMMO_NF * S;
    const int n16 = kObsFields * S;
    if ((S & 7) == 0) {
      const uint4* s4 = reinterpret_cast<const uint4*>(src);
      uint4* d4 = reinterpret_cast<uint4*>(T);
      for (int i = tid; i < n16 / 8; i += blockDim.x) d4[i] = s4[i];
    } else {
      for (int i = tid; i < n16; i += blockDim.x) T[i] = src[i];
    }
    for (int k = tid; k <= S; k += blockDim.x) rowpk[k] = 0xFFFFFFFFu;
  }
  __syncthreads();
  for (int s = tid; s < S; s += blockDim.x)
    if (T[F_ALIVE * S + s])
      rowpk[T[F_DS_ROW * S + s]] = (uint32_t)s | (uint32_t)(T[F_ROW * S + s] & 255) << 16 |
                                   (uint32_t)(T[F_COL * S + s] & 255) << 24;
  __syncthreads();

  const int lane = lane_id(), w = wave_id();
  int16_t* vis = vis_all + w * 128;
  uint2* inv = inv_all + w * kInv;
  const uint8_t* mat = p.mat + (size_t)e * kTiles;
  const int tick = p.env[(size_t)e * NMMO_NE + E_TICK];
  MaskCtx m;
  m.combat = (p.systems & NMMO_SYS_COMBAT) != 0;
  m.item = (p.systems & NMMO_SYS_ITEM) != 0;
  m.exch = m.item && (p.systems & NMMO_SYS_EXCHANGE) != 0;
  m.no_give = kWrap && (p.wflags & kWrapObsNoGive);
  // this wave's agents: a_j = g * 16 + w + 4 j; lane j holds a_j's task index and (wrapper) last
  // Sell price, loaded before any store
  constexpr int kPerWave = kFlatAgents / kFlatWaves;
  const int abase = g * kFlatAgents + w;
  int my_task = 0, my_prev = -1;
  // the row's state (ObsParams::zrow / zst): its Entity rows >= hv, its Market rows and
  // Buy.MarketItem entries >= hm are zero already (my_h = hv | hm << 12; a row of unknown content:
  // nothing is known zero, an all-zero row: everything)
  int my_h = kNObs | NMMO_MARKET_ROWS << 12;
  bool zv = false, zz = false, zt = false;
  if (lane < kPerWave && abase + kFlatWaves * lane < p.P) {
    const size_t ai = (size_t)e * p.P + abase + kFlatWaves * lane;
    my_task = p.assign[ai];
    if (p.ztag && p.zrow[ai] == p.ztag) {
      const uint64_t zs = p.zst[ai];
      zv = true;
      zz = (zs & kZsZero) != 0;
      zt = !zz && zs_task(zs) == my_task;
      my_h = zz ? 0 : zs_hv(zs) | zs_hm(zs) << 12;
    }
    if constexpr (kWrap)
      if (p.ws) my_prev = p.ws[ai].prev_price;
  }
  // bit j: agent j's row state describes this buffer / the row is all-zero / its Task section
  // holds agent j's task embedding already
  const uint64_t zvalid = __ballot(zv), zzero = __ballot(zz), zknown_task = __ballot(zt);
  auto task_known = [&](int j) { return ((zknown_task >> j) & 1) != 0; };
  int nrows = 0;             // rows this wave wrote (rows_out[0])
  unsigned long long nbytes = 0;  // bytes this wave stored (rows_out[1])
  // Entity.Query.window: ascending datastore rows within L-inf <= 7, first 100 -> vis, returns nv
  auto compact = [&](int r, int c) {
    int nv = 0;
    for (int base = 1; base <= S; base += 64) {
      const int k = base + lane;
      bool v = false;
      int q = -1;
      if (k <= S) {  // one LDS read per datastore row (its slot, row and column packed)
        const uint32_t wd = rowpk[k];
        q = (int)(wd & 0xFFFFu);
        v = wd != 0xFFFFFFFFu && linf(r, c, (int)((wd >> 16) & 255u), (int)(wd >> 24)) <= kVision;
      }
      const uint64_t b = __ballot(v);
      const int pos = nv + __popcll(b & lanes_below());
      if (v && pos < kNObs) vis[pos] = (int16_t)q;
      nv += __popcll(b);
    }
    return min(nv, kNObs);
  };
  // the agent's global loads: 12 item words (lanes 0..11), the 15x15 window materials (tile
  // lane + 64 i in wm[i]) and, for flat rows, the first kTaskRegs * 64 Task embedding floats
  uint2 iv;
  uint32_t wm[4];
  float tv[kTaskRegs > 0 ? kTaskRegs : 1];
  // the first kTaskRegs * 64 Task floats prefetched
  const bool treg = kTaskRegs > 0 && p.task_dim >= kTaskRegs * 64;
  uint8_t* wmat = wmat_all + w * 256;
  auto prefetch = [&](int a, int j) {
    const int r = T[F_ROW * S + a], c = T[F_COL * S + a];
    iv = lane < kInv ? p.items[((size_t)e * p.P + a) * kInv + lane] : make_uint2(0u, 0u);
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int t = lane + 64 * i;
      wm[i] = t < 225 ? mat[(r + t / 15 - kVision) * kSize + c + t % 15 - kVision] : 0u;
    }
    if (treg && !task_known(j)) {
      const float* temb = p.task + (size_t)__builtin_amdgcn_readlane(my_task, j) * p.task_dim + lane;
#pragma unroll
      for (int i = 0; i < kTaskRegs; i++) tv[i] = temb[64 * i];
    }
  };
  auto alive = [&](int j) {
    const int a = abase + kFlatWaves * j;
    return j < kPerWave && a < p.P && T[F_ALIVE * S + a] != 0;
  };
  if (alive(0)) prefetch(abase, 0);

  for (int j = 0; j < kPerWave; j++) {
    const int a = abase + kFlatWaves * j;
    if (a >= p.P) break;
    float* row = p.obs + ((size_t)e * p.P + a) * p.elems;
    const bool zv = (zvalid >> j) & 1;
    const int hj = __builtin_amdgcn_readlane(my_h, j);
    const int hv = hj & 4095, hm = hj >> 12;
    if (!T[F_ALIVE * S + a]) {  // not in the realm: an all-zero row
      if (alive(j + 1)) prefetch(a + kFlatWaves, j + 1);  // ahead of this row's stores
      if ((zzero >> j) & 1) continue;  // zeroed by an earlier launch into this buffer
      if (zv) {  // zero what the last write left nonzero
        wave_zero(row, 0, p.o_entity + hv * NMMO_N_ENTITY_COLS);
        wave_zero(row, p.o_inventory, p.o_market + hm * 16);
        wave_zero(row, p.o_task, p.elems);
        nbytes += 4ull * (p.o_entity + hv * NMMO_N_ENTITY_COLS + p.o_market + hm * 16 - p.o_inventory +
                          p.elems - p.o_task);
      } else {
        wave_zero(row, 0, p.elems);
        nbytes += 4ull * p.elems;
      }
      if (p.ztag && lane == 0) {
        p.zrow[(size_t)e * p.P + a] = p.ztag;
        p.zst[(size_t)e * p.P + a] = kZsZero;
      }
      nrows++;
      continue;
    }
    nrows++;
    const bool tknown = task_known(j);
    m.a = a;
    m.r = T[F_ROW * S + a];
    m.c = T[F_COL * S + a];
    m.gold = T[F_GOLD * S + a];
    // Tile: (row, column, material) per window tile; the materials go through LDS so the
    // prefetch registers are free before the compaction
#pragma unroll
    for (int i = 0; i < 4; i++)
      if (lane + 64 * i < 225) wmat[lane + 64 * i] = (uint8_t)wm[i];
    m.movebits = move_bits(wm[1]);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    // lane-per-tile: three dword stores 12 B apart per window tile (the pass's three stores fill
    // the same 768 bytes; measured 0.174 vs 0.196 ms per launch against contiguous stores with the
    // index arithmetic, and equal to one 12-B store, which costs the wrapper variant a VGPR over
    // the 4-wave limit)
#pragma unroll 1
    for (int t = lane; t < 225; t += 64) {
      const int tr = (t * 0x1112u) >> 16;  // t / 15 for t < 225
      float* d = &row[p.o_tile + 3 * t];
      obs_st(&d[0], (float)(m.r + tr - kVision));
      obs_st(&d[1], (float)(m.c + t - 15 * tr - kVision));
      obs_st(&d[2], (float)wmat[t]);
    }
    m.nv = compact(m.r, m.c);
    if (lane < kInv) inv[lane] = iv;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    m.ninv = inv_count(inv);
    m.prev_price = kWrap ? __builtin_amdgcn_readlane(my_prev, j) : -1;
    const int aid = T[F_ID * S + a];
    // Task (from registers; a task_dim beyond kTaskRegs * 64 reads the rest directly), unless the
    // row holds this task's embedding already
    if (!tknown) {
      nbytes += 4ull * p.task_dim;
      const int k0 = treg ? kTaskRegs * 64 : 0;  // a shorter embedding is read in place
      if (treg) {
        float* dst = row + p.o_task + lane;
#pragma unroll
        for (int i = 0; i < kTaskRegs; i++) obs_st(&dst[64 * i], tv[i]);
      }
      const float* temb = p.task + (size_t)__builtin_amdgcn_readlane(my_task, j) * p.task_dim;
      for (int k = k0 + lane; k < p.task_dim; k += 64) obs_st(&row[p.o_task + k], temb[k]);
    }
    // the next agent's loads go out now, ahead of this row's remaining stores
    if (alive(j + 1)) prefetch(a + kFlatWaves, j + 1);
    // ActionTargets, section by section
    mask_sec_f32<0, kWrap>(p, T, S, vis, inv, mpo, nm, m, row);
    mask_sec_f32<1, kWrap>(p, T, S, vis, inv, mpo, nm, m, row);
    {  // Buy.MarketItem: the listings' entries, the zero entries up to hm, and the no-op entry
      const int n = max(nm, hm);
      for (int k = lane; k < n; k += 64)
        obs_st(&row[p.o_buy + k], mask_value<kWrap>(p, T, S, vis, inv, mpo, nm, m, 2, k) ? 1.f : 0.f);
      if (lane == 0) obs_st(&row[p.o_buy + NMMO_MARKET_ROWS], 1.f);
      nbytes += 4ull * (p.o_agent_id + 2 - NMMO_MARKET_ROWS + n);  // every mask but Buy's tail, id, tick
    }
    mask_sec_f32<3, kWrap>(p, T, S, vis, inv, mpo, nm, m, row);
    mask_sec_f32<4, kWrap>(p, T, S, vis, inv, mpo, nm, m, row);
    mask_sec_f32<5, kWrap>(p, T, S, vis, inv, mpo, nm, m, row);
    mask_sec_f32<6, kWrap>(p, T, S, vis, inv, mpo, nm, m, row);
    mask_sec_f32<7, kWrap>(p, T, S, vis, inv, mpo, nm, m, row);
    mask_sec_f32<8, kWrap>(p, T, S, vis, inv, mpo, nm, m, row);
    mask_sec_f32<9, kWrap>(p, T, S, vis, inv, mpo, nm, m, row);
    mask_sec_f32<10, kWrap>(p, T, S, vis, inv, mpo, nm, m, row);
    mask_sec_f32<11, kWrap>(p, T, S, vis, inv, mpo, nm, m, row);
    if (lane == 0) obs_st(&row[p.o_agent_id], (float)aid);
    if (lane == 1) obs_st(&row[p.o_tick], (float)tick);
    // Entity rows: two per pass (lanes 0-30 row k, lanes 32-62 row k + 1: 62 contiguous floats),
    // the rows past the visible ones as one zero run
    {
      const int f = lane & 31, half = lane >> 5;
      const int nv2 = (m.nv + 1) & ~1;
#pragma unroll 1
      for (int k0 = 0; k0 < nv2; k0 += 2) {
        const int k = k0 + half;
        if (f < NMMO_N_ENTITY_COLS)
          obs_st(&row[p.o_entity + k * NMMO_N_ENTITY_COLS + f], k < m.nv ? (float)T[f * S + vis[k]] : 0.f);
      }
      const int hz = max(nv2, hv);  // the rows past the visible ones not known zero
      wave_zero(row, p.o_entity + nv2 * NMMO_N_ENTITY_COLS, p.o_entity + hz * NMMO_N_ENTITY_COLS);
      nbytes += 4ull * (hz * NMMO_N_ENTITY_COLS + kInv * 16 + max(nm, hm) * 16 + 225 * 3);
      if (p.ztag && lane == 0) {
        if (!zv) p.zrow[(size_t)e * p.P + a] = p.ztag;
        p.zst[(size_t)e * p.P + a] = zs_pack(nv2, nm, __builtin_amdgcn_readlane(my_task, j));
      }
    }
    // Inventory (own items, owner = self) and Market (env listings, ascending row)
    for (int k = lane; k < kInv * 16; k += 64) {
      const int q = k >> 4;
      obs_st(&row[p.o_inventory + k], q < m.ninv ? item_col(inv[q], aid, k & 15) : 0.f);
    }
    for (int k = lane; k < nm * 16; k += 64)
      obs_st(&row[p.o_market + k], item_col(mitem[k >> 4], (mpo[k >> 4] >> 8) + 1, k & 15));
    wave_zero(row, p.o_market + nm * 16, p.o_market + max(nm, hm) * 16);
    __builtin_amdgcn_wave_barrier();
  }
  if (p.rows_out && lane == 0 && nrows) {  // per env: one address per env keeps the atomics uncontended
    atomicAdd(&p.rows_out[2 * e], (unsigned long long)nrows);
    atomicAdd(&p.rows_out[2 * e + 1], nbytes);
  }
}

hipError_t launch_obs(const ObsParams& p, hipStream_t stream) {
  if (p.wire) return launch_wire_obs(p, stream);  // wire_obs.hip
  if (p.nat) return launch_native_obs(p, stream);  // native_obs.hip
  const int ne = list_grid(p.env_list, p.n_list, p.n_envs);
  if (ne <= 0) return hipSuccess;
#ifdef NMMO_OBS_XCD
  const dim3 grid(ne * ((p.P + kFlatAgents - 1) / kFlatAgents)), block(64 * kFlatWaves);
#else
  const dim3 grid(ne, (p.P + kFlatAgents - 1) / kFlatAgents), block(64 * kFlatWaves);
#endif
  const size_t lds = obs_lds_bytes(p.S);
  if (p.ztag) {  // the bound buffer: incremental rows (flat_obs.hip; here the round-4 kernel for slot
                 // counts that are not a multiple of 8, and under NMMO_FLAT_V1)
#ifndef NMMO_FLAT_V1
    if (flat_obs_ok(p)) return launch_flat_obs(p, stream);
#endif
    if (p.wflags) hipLaunchKernelGGL((obs_kernel<true, false>), grid, block, lds, stream, p);
    else hipLaunchKernelGGL((obs_kernel<false, false>), grid, block, lds, stream, p);
  } else {  // every row in full
    if (p.wflags) hipLaunchKernelGGL((obs_kernel<true, true>), grid, block, lds, stream, p);
    else hipLaunchKernelGGL((obs_kernel<false, true>), grid, block, lds, stream, p);
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------- native -> flat (SPEC §8b)
// For learners that want pufferlib's float32 row from the native layout (e.g. after gathering
// native shards over xGMI). Grid (env, 16-agent group), 4 waves; the env's Market (32 KB) is
// staged in LDS once per workgroup; one wave expands one agent row. HBM-write-bound like
// obs_kernel: 95,948 B written per agent for 9,552 B (+ 1/16 of the Market) read.
__global__ void __launch_bounds__(256) expand_kernel(ObsParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  int16_t* mk = reinterpret_cast<int16_t*>(smem);
  const int e = blockIdx.x, g = blockIdx.y, tid = threadIdx.x;
  const uint8_t* base = p.nat + (size_t)e * native_env_bytes(p.P);
  {
    const uint4* src = reinterpret_cast<const uint4*>(base + (size_t)p.P * NMMO_NATIVE_ROW_BYTES);
    uint4* dst = reinterpret_cast<uint4*>(mk);
    for (int i = tid; i < NMMO_NATIVE_MARKET_BYTES / 16; i += blockDim.x) dst[i] = src[i];
  }
  __syncthreads();
  const int lane = lane_id(), w = wave_id();
  for (int i = w; i < kObsAgentsPerBlock; i += kObsWaves) {
    const int a = g * kObsAgentsPerBlock + i;
    if (a >= p.P) break;
    const uint8_t* nrow = base + (size_t)a * NMMO_NATIVE_ROW_BYTES;
    const int16_t* q = reinterpret_cast<const int16_t*>(nrow + NMMO_NATIVE_MASK_BYTES);
    const int frow = p.row_map ? p.row_map[(size_t)e * p.P + a] : e * p.P + a;
    if (frow < 0) continue;  // storage: row not kept (wave-uniform)
    float* row = p.obs + (size_t)frow * p.elems;
    const int aid = __builtin_amdgcn_readfirstlane(q[0]);
    if (aid == 0) {  // not in the realm: all-zero row
      wave_zero(row, 0, p.elems);
      continue;
    }
    for (int j = lane; j < p.o_agent_id; j += 64) obs_st(&row[j], (float)nrow[j]);
    if (lane == 0) obs_st(&row[p.o_agent_id], (float)aid);
    if (lane == 1) obs_st(&row[p.o_tick], (float)q[1]);
    for (int j = lane; j < kNObs * NMMO_N_ENTITY_COLS; j += 64) obs_st(&row[p.o_entity + j], (float)q[kNatEntity + j]);
    for (int j = lane; j < kInv * 16; j += 64) obs_st(&row[p.o_inventory + j], (float)q[kNatInv + j]);
    for (int j = lane; j < NMMO_MARKET_ROWS * 16; j += 64) obs_st(&row[p.o_market + j], (float)mk[j]);
    const float* temb = p.task + (size_t)q[kNatTask] * p.task_dim;
    for (int j = lane; j < p.task_dim; j += 64) obs_st(&row[p.o_task + j], temb[j]);
    for (int j = lane; j < 225 * 3; j += 64) obs_st(&row[p.o_tile + j], (float)q[kNatTile + j]);
    __builtin_amdgcn_wave_barrier();
  }
}

hipError_t launch_expand(const ObsParams& p, hipStream_t stream) {
  dim3 grid(p.n_envs, (p.P + kObsAgentsPerBlock - 1) / kObsAgentsPerBlock);
  hipLaunchKernelGGL(expand_kernel, grid, dim3(64 * kObsWaves), NMMO_NATIVE_MARKET_BYTES, stream, p);
  return hipGetLastError();
}

// ---------------------------------------------------------------- scripted policy (SPEC §10)
// One workgroup per env: for every head, a uniform draw over the set bits of that head's mask
// (identical to the obs masks). Phase A: alive entities are bucketed into a uniform grid of
// 16x16-tile cells; each player (thread) tests the entities of the <= 2x2 cells its window
// touches and sets its visible / attackable / same-tile row bits. Phase B (thread per player):
// the first-100-visible cut, counts, draws and k-th-set-bit selections with popcounts.
__host__ __device__ inline int policy_threads(int S, int P) {
  const int t = ((S + 63) / 64) * 64;
  return t < P ? ((P + 63) / 64) * 64 : t;
}
__host__ __device__ inline size_t policy_lds_bytes(int S, int P) {
  const int NW = (S + 63) / 64;
  const size_t b = (size_t)3 * P * NW * 8 + (size_t)((P + 3) & ~3) * 4 + (size_t)NMMO_MARKET_ROWS * 12;
  return ((b + 15) & ~(size_t)15) + grid_lds_bytes(S);
}

__device__ __forceinline__ void policy_body(const PolicyParams& p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int S = p.S, P = p.P, e = blockIdx.x, tid = threadIdx.x;
  const int NW = (S + 63) >> 6;
  uint64_t* vism = reinterpret_cast<uint64_t*>(smem);  // [P][NW] visible rows
  uint64_t* atkm = vism + P * NW;                      // [P][NW] attackable rows
  uint64_t* samm = atkm + P * NW;                      // [P][NW] other players on the same tile
  uint32_t* ppos = reinterpret_cast<uint32_t*>(samm + P * NW);  // [P] r<<16 | c, or sentinel
  uint2* mitem = reinterpret_cast<uint2*>(ppos + ((P + 3) & ~3));
  int* mown = reinterpret_cast<int*>(mitem + NMMO_MARKET_ROWS);
  // grid (common.h; grid_lds_bytes): cell -> first entry, entries
  unsigned char* gb = smem + ((reinterpret_cast<unsigned char*>(mown + NMMO_MARKET_ROWS) - smem + 15) & ~15);
  int* gstart = reinterpret_cast<int*>(gb);
  uint32_t* glist = reinterpret_cast<uint32_t*>(gb + (((kGridCells + 1) * 4 + 15) & ~15));
  const int16_t* E = p.ent + (size_t)e * NMMO_NF * S;
  const bool combat = (p.systems & NMMO_SYS_COMBAT) != 0;
  const bool item = (p.systems & NMMO_SYS_ITEM) != 0;
  const bool exch = item && (p.systems & NMMO_SYS_EXCHANGE) != 0;
  const int nm = exch ? p.mcount[e] : 0;
  for (int j = tid; j < nm; j += blockDim.x) {
    const int v = p.mlist[(size_t)e * NMMO_MARKET_ROWS + j];
    mown[j] = (v >> 16) & 255;
    mitem[j] = p.items[((size_t)e * P + ((v >> 16) & 255)) * kInv + ((v >> 24) & 15)];
  }
  for (int a = tid; a < ((P + 3) & ~3); a += blockDim.x)
    ppos[a] = (a < P && E[F_ALIVE * S + a]) ? ((uint32_t)E[F_ROW * S + a] << 16) | (uint32_t)E[F_COL * S + a]
                                            : 0x80008000u;
  const bool tgt_any = combat || item;
  if (tgt_any) {
    uint32_t* m32 = reinterpret_cast<uint32_t*>(vism);  // vism | atkm | samm, contiguous
    for (int k = tid; k < 6 * P * NW; k += blockDim.x) m32[k] = 0;
    // grid entry: (ds_row-1)<<16 | r<<8 | c, bit 30 = not spawn-immune (players)
    int cell = -1;
    uint32_t gv = 0;
    if (tid < S && E[F_ALIVE * S + tid]) {  // policy_threads >= S
      const int r = E[F_ROW * S + tid], c = E[F_COL * S + tid];
      const bool pl = tid < P, immune = pl && E[F_TIME_ALIVE * S + tid] < p.spawn_immunity;
      cell = (pl ? 0 : kCells) + (r >> kCellShift) * kGrid + (c >> kCellShift);
      gv = ((uint32_t)(E[F_DS_ROW * S + tid] - 1) << 16) | (uint32_t)(r << 8) | (uint32_t)c |
           (immune ? 0u : 1u << 30);
    }
    grid_build(gstart, glist, cell, gv);  // its barriers also cover ppos and m32
    // kWinRows threads per player, one grid row of its window each; no-return LDS atomics
    for (int t = tid; t < kWinRows * P; t += blockDim.x) {
      const int a = t / kWinRows;
      if (ppos[a] == 0x80008000u) continue;
      const int r = (int)(ppos[a] >> 16), c = (int)(ppos[a] & 0xFFFF);
      const int4 wdw = grid_window(r, c);
      const int cr = wdw.x + (t - kWinRows * a);
      if (cr > wdw.y) continue;
      uint32_t* mv = reinterpret_cast<uint32_t*>(vism + a * NW);
      uint32_t* ma = reinterpret_cast<uint32_t*>(atkm + a * NW);
      uint32_t* ms = reinterpret_cast<uint32_t*>(samm + a * NW);
      const int g = cr * kGrid;
      grid_scan(glist, gstart[g + wdw.z], gstart[g + wdw.w + 1], r, c, [&](uint32_t v, int d, int) {
        const int wi = (v >> 21) & 15;  // players: visible, attackable unless immune, same tile
        const uint32_t bit = 1u << ((v >> 16) & 31);
        atomicOr(&mv[wi], bit);
        if (d <= 3 && (v & (1u << 30))) atomicOr(&ma[wi], bit);
        if (d == 0) atomicOr(&ms[wi], bit);
      });
      grid_scan(glist, gstart[kCells + g + wdw.z], gstart[kCells + g + wdw.w + 1], r, c,
                [&](uint32_t v, int d, int) {  // NPCs: visible, attackable
                  const int wi = (v >> 21) & 15;
                  const uint32_t bit = 1u << ((v >> 16) & 31);
                  atomicOr(&mv[wi], bit);
                  if (d <= 3) atomicOr(&ma[wi], bit);
                });
    }
  }
  __syncthreads();
  for (int a = tid; a < P && tgt_any; a += blockDim.x) {  // a player never targets itself
    if (!E[F_ALIVE * S + a]) continue;
    const int r0 = E[F_DS_ROW * S + a] - 1;
    atkm[a * NW + (r0 >> 6)] &= ~(1ull << (r0 & 63));
    samm[a * NW + (r0 >> 6)] &= ~(1ull << (r0 & 63));
  }
  __syncthreads();
  const int32_t* env = p.env + (size_t)e * NMMO_NE;
  const uint8_t* mat = p.mat + (size_t)e * kTiles;
  for (int a = tid; a < P; a += blockDim.x) {
    int32_t* out = p.actions + ((size_t)e * P + a) * kHeads;
    int32_t h[kHeads] = {0, kNObs, NMMO_MARKET_ROWS, kInv, kInv, kNObs, 0, kNObs, 0, kInv, 0, kInv};
    if (!E[F_ALIVE * S + a]) {
#pragma unroll
      for (int k = 0; k < kHeads; k++) out[k] = 0;
      continue;
    }
    const uint32_t c0 = (uint32_t)env[E_TICK] + 2048u * (uint32_t)env[E_EPISODE];
    const uint32_t c1 = (uint32_t)env[E_ENV_INDEX];
    const uint32_t k0 = (uint32_t)p.seed, k1 = (uint32_t)(p.seed >> 32);
    // U(u, 1) = 0 for every u: a head with one legal index needs no Philox call (exact)
    auto draw_n = [&](int head, int n) {
      return n <= 1 ? 0 : (int)uniform_n(philox(c0, c1, (uint32_t)a, (uint32_t)head, k0, k1).x, (uint32_t)n);
    };
    const int r = E[F_ROW * S + a], c = E[F_COL * S + a], gold = E[F_GOLD * S + a];
    if (combat) h[0] = draw_n(0, 3);
    if (tgt_any) {
      // Entity rows beyond the first 100 visible are not in the obs: cut the masks there
      int na = 0, nt = 0, cum = 0;
      for (int w = 0; w < NW; w++) {
        uint64_t cut = vism[a * NW + w];
        const int pc = __popcll(cut);
        if (cum + pc > kNObs) {
          for (int i = 0; i < cum + pc - kNObs; i++) cut &= ~(1ull << (63 - __builtin_clzll(cut)));
        }
        cum = min(cum + pc, kNObs);
        na += __popcll(atkm[a * NW + w] & cut);
        nt += __popcll(samm[a * NW + w] & cut);
      }
      const int pa = combat ? draw_n(1, na + 1) : na;
      const int pg = draw_n(5, (item ? nt : 0) + 1);
      const int pgg = draw_n(7, (exch ? nt : 0) + 1);
      // visible index of the k-th set bit of mask m (within the cut)
      auto select = [&](const uint64_t* m, int k) {
        int before = 0;
        for (int w = 0; w < NW; w++) {
          const uint64_t vm = vism[a * NW + w];
          uint64_t mm = m[a * NW + w] & vm;
          const int pc = __popcll(mm);
          if (k < pc) {
            for (int i = 0; i < k; i++) mm &= mm - 1;
            const int b = __builtin_ctzll(mm);
            return before + (int)__popcll(vm & ((1ull << b) - 1ull));
          }
          k -= pc;
          before += (int)__popcll(vm);
        }
        return (int)kNObs;
      };
      if (combat && pa < na) h[1] = select(atkm, pa);
      if (item && pg < nt) h[5] = select(samm, pg);
      if (exch && pgg < nt) h[7] = select(samm, pgg);
    }
    // Buy.MarketItem: listings with price <= gold not owned by self
    {
      int nb = 0;
      for (int j = 0; j < nm; j++) nb += it_price(mitem[j]) <= gold && mown[j] != a;
      const int pick = draw_n(2, nb + 1);
      int sel = NMMO_MARKET_ROWS;
      for (int j = 0, seen = 0; j < nm && sel == NMMO_MARKET_ROWS; j++) {
        const bool ok = it_price(mitem[j]) <= gold && mown[j] != a;
        sel = (ok && seen == pick) ? j : sel;
        seen += ok;
      }
      h[2] = sel;
    }
    // InventoryItem heads: Destroy (3), Give (4), Sell (9), Use (11)
    {
      uint2 inv[kInv];
      const uint4* src = reinterpret_cast<const uint4*>(p.items + ((size_t)e * P + a) * kInv);
#pragma unroll
      for (int k = 0; k < kInv / 2; k++) {
        const uint4 q = item ? src[k] : make_uint4(0u, 0u, 0u, 0u);
        inv[2 * k] = make_uint2(q.x, q.y);
        inv[2 * k + 1] = make_uint2(q.z, q.w);
      }
      int nf = 0, ns = 0, nu = 0;
      uint32_t mf = 0, msl = 0, mu = 0;
#pragma unroll
      for (int k = 0; k < kInv; k++) {
        const uint2 w = inv[k];
        const bool present = it_type(w) != 0;
        const bool f = present && !it_equipped(w) && !it_price(w);
        const bool sl = present && !it_equipped(w);
        const bool us = present && item_usable(E, S, a, w);
        mf |= (uint32_t)f << k;
        msl |= (uint32_t)sl << k;
        mu |= (uint32_t)us << k;
      }
      if (!item) mf = mu = 0;
      if (!exch) msl = 0;
      nf = __popc(mf);
      ns = __popc(msl);
      nu = __popc(mu);
      auto kth = [](uint32_t m, int k) {
        for (int i = 0; i < k; i++) m &= m - 1;
        return (int)__builtin_ctz(m);
      };
      const int pd = draw_n(3, nf + 1), pgv = draw_n(4, nf + 1);
      const int ps = draw_n(9, ns + 1), pu = draw_n(11, nu + 1);
      h[3] = pd < nf ? kth(mf, pd) : kInv;
      h[4] = pgv < nf ? kth(mf, pgv) : kInv;
      h[9] = ps < ns ? kth(msl, ps) : kInv;
      h[11] = pu < nu ? kth(mu, pu) : kInv;
    }
    if (exch) {
      const int ng = min(gold, 99);
      h[6] = ng > 0 ? draw_n(6, ng) : 0;
      h[10] = draw_n(10, 99);
    }
    int mv[5], nmv = 0;
#pragma unroll
    for (int d = 0; d < 5; d++)
      if (!impassable(mat[(r + dir_dr(d)) * kSize + c + dir_dc(d)])) mv[nmv++] = d;
    h[8] = nmv ? mv[draw_n(8, nmv)] : 0;
#pragma unroll
    for (int k = 0; k < kHeads; k++) out[k] = h[k];
  }
}

__global__ void __launch_bounds__(512) policy_kernel(PolicyParams p) { policy_body(p); }
// <= 64 VGPRs / 96 SGPRs: a 6-wave workgroup (S = 384) puts two waves on two SIMDs, so 4 per CU
// need 8 wave slots there (C3/C4: 21 -> 17 us per launch; the 2-wave C2 launch is faster without)
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(8, 8))) policy_kernel_w8(PolicyParams p) {
  policy_body(p);
}

hipError_t launch_policy(const PolicyParams& p, hipStream_t stream) {
  if (p.S > 511) return hipErrorInvalidValue;  // grid entries hold ds_row - 1 in 9 bits
  const int threads = policy_threads(p.S, p.P);
  hipLaunchKernelGGL(threads > 256 ? policy_kernel_w8 : policy_kernel, dim3(p.n_envs), dim3(threads),
                     policy_lds_bytes(p.S, p.P), stream, p);
  return hipGetLastError();
}

}  // namespace nmmo
