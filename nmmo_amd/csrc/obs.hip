// obs.hip — per-agent observation gather (SPEC.md §8) and the scripted masked-uniform policy
// (SPEC.md §10).
//
// Replaces Env._compute_observations + pufferlib's flatten/pad (the buffer the reference
// receives from pool.recv(), clean_pufferl.py:293, and decodes with unpack_batched_obs,
// baseline_policy.py:41). Output: float32 [n_envs][P][23,987] in pufferlib sorted-key order.
//
// Roofline: this kernel is HBM-write-bound — 95,948 B written per agent row against ~0.3 KB of
// reads (the env's entity columns are staged once per workgroup in LDS and shared by its 16
// agents; the 225 map bytes per agent come from L2). One wave owns one agent row at a time:
// it compacts the agent's visible entities with a ballot/prefix-popcount over datastore rows
// (the nmmo window order) into LDS, then streams the row with coalesced stores — 16-byte
// stores for the long constant runs (Inventory+Market), dword stores elsewhere.
#include "kernels.h"

namespace nmmo {

constexpr int kObsAgentsPerBlock = 16;
constexpr int kObsWaves = 4;
constexpr int kObsFields = F_DS_ROW + 1;  // 0..30 obs columns, alive, ds_row

// LDS: entity fields | row->slot | per-wave visible list | per-wave inventory | market listings
// (flat: listed item words + owners, 12 B per listing; native: price | owner << 8, 2 B per listing,
// and per-wave 15x15 window materials)
__host__ __device__ inline size_t obs_lds_bytes(int S, bool native) {
  return (((size_t)kObsFields * S * 2 + 15) & ~(size_t)15) + (((size_t)(S + 1) * 2 + 15) & ~(size_t)15) +
         (size_t)kObsWaves * 128 * 2 + (size_t)kObsWaves * kInv * 8 +
         (native ? (size_t)NMMO_MARKET_ROWS * 2 + (size_t)kObsWaves * 256 : (size_t)NMMO_MARKET_ROWS * 12);
}

// Plain (temporal) stores. Measured on MI355X (same-box A/B): __builtin_nontemporal_store
// ("nt") made the C4 obs kernel 33% slower (3.52 vs 2.65 ms per launch); building every row
// from 16-byte stores (4 consecutive elements per lane) was 54% slower (3.25 vs 2.11 ms: the
// per-element section dispatch doubled the VGPRs and halved occupancy).
__device__ __forceinline__ void obs_st(float* p, float v) { *p = v; }
__device__ __forceinline__ void obs_st4(float4* p, float4 v) { *p = v; }

// zero [lo, hi) of a row with 16-byte stores on the aligned body (wave-cooperative)
__device__ inline void wave_zero(float* row, int lo, int hi) {
  const int lane = lane_id();
  const uintptr_t a = reinterpret_cast<uintptr_t>(row + lo);
  int head = (int)(((16 - (a & 15)) & 15) >> 2);
  if (head > hi - lo) head = hi - lo;
  if (lane < head) obs_st(&row[lo + lane], 0.f);
  const int body = (hi - lo - head) >> 2;
  float4* p4 = reinterpret_cast<float4*>(row + lo + head);
  for (int i = lane; i < body; i += 64) obs_st4(&p4[i], make_float4(0.f, 0.f, 0.f, 0.f));
  const int tail0 = lo + head + body * 4;
  if (tail0 + lane < hi) obs_st(&row[tail0 + lane], 0.f);
}

// native layout (SPEC §8b): int16 part offsets, env stride, two int16 per dword store
constexpr int kNatEntity = 2, kNatInv = kNatEntity + kNObs * NMMO_N_ENTITY_COLS,
              kNatTile = kNatInv + kInv * 16, kNatTask = kNatTile + 225 * 3;
static_assert(kNatTask < NMMO_NATIVE_I16, "native int16 part overflows its row");
__host__ __device__ inline size_t native_env_bytes(int P) {
  return (size_t)P * NMMO_NATIVE_ROW_BYTES + NMMO_NATIVE_MARKET_BYTES;
}
__device__ __forceinline__ uint32_t i16pack(int lo, int hi) {
  return (uint32_t)(uint16_t)(int16_t)lo | ((uint32_t)(uint16_t)(int16_t)hi << 16);
}

// kWrap: the wrapper's observation() edits are compiled in (SPEC §13). Both variants stay at
// 79 VGPRs = 6 waves/SIMD (a run-time flag check in the shared body cost 2 VGPRs and a wave).
// kNative: the nmmo-dtype layout of SPEC §8b (u8 masks, int16 fields, Market once per env,
// task index) instead of pufferlib's float32 row: ~10x fewer bytes per agent.
template <bool kWrap, bool kNative>
__global__ void __launch_bounds__(256) obs_kernel(ObsParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int S = p.S;
  int16_t* T = reinterpret_cast<int16_t*>(smem);
  int16_t* rowslot = reinterpret_cast<int16_t*>(smem + (((size_t)kObsFields * S * 2 + 15) & ~(size_t)15));
  int16_t* vis_all = rowslot + ((((size_t)(S + 1) * 2 + 15) & ~(size_t)15) / 2);
  uint2* inv_all = reinterpret_cast<uint2*>(vis_all + kObsWaves * 128);
  uint2* mitem = inv_all + kObsWaves * kInv;                       // flat: listed item words
  int* mown = reinterpret_cast<int*>(mitem + NMMO_MARKET_ROWS);    // flat: listing owner slot
  uint16_t* mpo = reinterpret_cast<uint16_t*>(inv_all + kObsWaves * kInv);  // native: price | owner << 8
  uint8_t* wmat_all = reinterpret_cast<uint8_t*>(mpo + NMMO_MARKET_ROWS);   // native only
  const int e = blockIdx.x, g = blockIdx.y;
  const int tid = threadIdx.x;
  const int nm = p.mcount[e];
  for (int j = tid; j < nm; j += blockDim.x) {  // end-of-tick listings, ascending row
    const int v = p.mlist[(size_t)e * NMMO_MARKET_ROWS + j];
    const int own = (v >> 16) & 255, slot = (v >> 24) & 15;
    const uint2 wd = p.items[((size_t)e * p.P + own) * kInv + slot];
    if constexpr (kNative) {
      mpo[j] = (uint16_t)(it_price(wd) | own << 8);
    } else {
      mown[j] = own;
      mitem[j] = wd;
    }
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
    for (int k = tid; k <= S; k += blockDim.x) rowslot[k] = -1;
  }
  __syncthreads();
  for (int s = tid; s < S; s += blockDim.x)
    if (T[F_ALIVE * S + s]) rowslot[T[F_DS_ROW * S + s]] = (int16_t)s;
  __syncthreads();

  if constexpr (kNative) {  // the env's Market, once per env (the y == 0 workgroup)
    if (g == 0) {  // one listing row (16 int16 = two 16-B stores) per thread
      uint4* mk = reinterpret_cast<uint4*>(p.nat + (size_t)e * native_env_bytes(p.P) +
                                           (size_t)p.P * NMMO_NATIVE_ROW_BYTES);
      for (int k = tid; k < NMMO_MARKET_ROWS; k += blockDim.x) {
        uint32_t q[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
        if (k < nm) {
          const int v = p.mlist[(size_t)e * NMMO_MARKET_ROWS + k];
          const int own = (v >> 16) & 255, slot = (v >> 24) & 15;
          const uint2 wd = p.items[((size_t)e * p.P + own) * kInv + slot];
#pragma unroll
          for (int i = 0; i < 8; i++)
            q[i] = i16pack((int)item_col(wd, own + 1, 2 * i), (int)item_col(wd, own + 1, 2 * i + 1));
        }
        mk[2 * k] = make_uint4(q[0], q[1], q[2], q[3]);
        mk[2 * k + 1] = make_uint4(q[4], q[5], q[6], q[7]);
      }
    }
  }
  const int lane = lane_id(), w = wave_id();
  int16_t* vis = vis_all + w * 128;
  uint8_t* wmat = wmat_all + w * 256;
  const uint8_t* mat = p.mat + (size_t)e * kTiles;
  const int tick = p.env[(size_t)e * NMMO_NE + E_TICK];
  const bool combat = (p.systems & NMMO_SYS_COMBAT) != 0;
  const bool item = (p.systems & NMMO_SYS_ITEM) != 0;
  const bool exch = item && (p.systems & NMMO_SYS_EXCHANGE) != 0;
  uint2* inv = inv_all + w * kInv;
  for (int i = w; i < kObsAgentsPerBlock; i += kObsWaves) {
    const int a = g * kObsAgentsPerBlock + i;
    if (a >= p.P) break;
    float* row = kNative ? nullptr : p.obs + ((size_t)e * p.P + a) * p.elems;
    uint8_t* nrow = kNative ? p.nat + (size_t)e * native_env_bytes(p.P) + (size_t)a * NMMO_NATIVE_ROW_BYTES : nullptr;
    if (!T[F_ALIVE * S + a]) {
      if constexpr (kNative) {
        uint4* z = reinterpret_cast<uint4*>(nrow);
        for (int j = lane; j < NMMO_NATIVE_ROW_BYTES / 16; j += 64) z[j] = make_uint4(0u, 0u, 0u, 0u);
      } else {
        wave_zero(row, 0, p.elems);
      }
      continue;
    }
    const int r = T[F_ROW * S + a], c = T[F_COL * S + a];
    const int gold = T[F_GOLD * S + a];
    if (lane < kInv) inv[lane] = p.items[((size_t)e * p.P + a) * kInv + lane];
    uint32_t wm[4] = {0u, 0u, 0u, 0u};  // native: the 15x15 window materials, tile lane + 64 i
    if constexpr (kNative) {
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int t = lane + 64 * i;
        if (t < 225) wm[i] = mat[(r + t / 15 - kVision) * kSize + c + t % 15 - kVision];
      }
    }
    // Entity.Query.window: ascending datastore rows within L-inf <= 7, first 100
    int nv = 0;
    for (int base = 1; base <= S; base += 64) {
      const int k = base + lane;
      bool v = false;
      int q = -1;
      if (k <= S) {
        q = rowslot[k];
        v = q >= 0 && linf(r, c, T[F_ROW * S + q], T[F_COL * S + q]) <= kVision;
      }
      const uint64_t b = __ballot(v);
      const int pos = nv + __popcll(b & lanes_below());
      if (v && pos < kNObs) vis[pos] = (int16_t)q;
      nv += __popcll(b);
    }
    nv = min(nv, kNObs);
    if constexpr (kNative) {
#pragma unroll
      for (int i = 0; i < 4; i++)
        if (lane + 64 * i < 225) wmat[lane + 64 * i] = (uint8_t)wm[i];
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");

    const int ninv = inv_count(inv);
    const int prev_price = kWrap && p.ws ? __builtin_amdgcn_readfirstlane(p.ws[(size_t)e * p.P + a].prev_price) : -1;
    const int aid = T[F_ID * S + a];
    // ActionTargets [0, o_agent_id) (SPEC §8, §9)
    auto mask_val = [&](int j) -> bool {
      bool v = false;
      if (j < p.o_target) {
        v = combat;
      } else if (j < p.o_buy) {
        const int k = j - p.o_target;
        if (k == kNObs) v = true;
        else if (combat && k < nv) {
          const int q = vis[k];
          v = q != a && linf(r, c, T[F_ROW * S + q], T[F_COL * S + q]) <= 3 &&
              !(q < p.P && T[F_TIME_ALIVE * S + q] < p.spawn_immunity);
        }
      } else if (j < p.o_destroy) {
        const int k = j - p.o_buy;
        v = k == NMMO_MARKET_ROWS || (exch && k < nm && it_price(mitem[k]) <= gold && mown[k] != a);
      } else if (j < p.o_give_target) {  // Destroy.InventoryItem, Give.InventoryItem
        const int k = j < p.o_give_item ? j - p.o_destroy : j - p.o_give_item;
        v = k == kInv || (item && k < ninv && !it_equipped(inv[k]) && !it_price(inv[k]));
      } else if (j < p.o_gg_price || (j >= p.o_gg_target && j < p.o_move)) {  // Give/GiveGold.Target
        const bool on = j < p.o_gg_price ? item : exch;
        const int k = j < p.o_gg_price ? j - p.o_give_target : j - p.o_gg_target;
        if (k == kNObs) v = true;
        else if (on && k < nv) {
          const int q = vis[k];
          v = q < p.P && q != a && T[F_ROW * S + q] == r && T[F_COL * S + q] == c;
        }
      } else if (j < p.o_gg_target) {
        v = exch && j - p.o_gg_price < gold;
      } else if (j < p.o_sell_item) {
        const int d = j - p.o_move;
        v = !impassable(mat[(r + dir_dr(d)) * kSize + c + dir_dc(d)]);
      } else if (j < p.o_sell_price) {
        const int k = j - p.o_sell_item;
        v = k == kInv || (exch && k < ninv && !it_equipped(inv[k]));
      } else if (j < p.o_use) {
        v = exch;
      } else {
        const int k = j - p.o_use;
        v = k == kInv || (item && k < ninv && item_usable(T, S, a, inv[k]));
      }
      if constexpr (kWrap) {  // wrapper observation() edits (SPEC §13)
        if ((p.wflags & kWrapObsPrice) && j >= p.o_sell_price && j < p.o_use && j - p.o_sell_price == prev_price)
          v = false;
        if ((p.wflags & kWrapObsNoGive) && j >= p.o_give_item && j < p.o_move) {
          const bool keep = j == p.o_give_target - 1 || j == p.o_gg_price - 1 || j == p.o_gg_price ||
                            j == p.o_move - 1;  // Give.InventoryItem/Target noop, Price 0, GiveGold noop
          if (!keep) v = false;
        }
        if ((p.wflags & kWrapObsNoDangerous) && j >= p.o_target && j < p.o_buy) {
          const int k = j - p.o_target;
          if (k < nv && T[F_NPC_TYPE * S + vis[k]] > 1) v = false;
        }
      }
      return v;
    };
    if constexpr (kNative) {
      // Section by section (no per-element section dispatch): every lane of a store works on the
      // same section, the window materials were prefetched into registers ahead of the
      // visibility compaction, and nothing below waits on global memory.
      uint8_t* mb = nrow;  // u8 ActionTargets in flat order, then pad to NMMO_NATIVE_MASK_BYTES
      const bool no_give = kWrap && (p.wflags & kWrapObsNoGive);
      auto free_item = [&](int k) { return k < ninv && !it_equipped(inv[k]) && !it_price(inv[k]); };
      auto same_tile = [&](int k) {
        const int q = vis[k];
        return q < p.P && q != a && T[F_ROW * S + q] == r && T[F_COL * S + q] == c;
      };
      // Buy.MarketItem (1,025 entries, the longest section): four entries per lane per dword store
      // from one 8-B LDS read of the packed listings (the section starts dword-aligned in the
      // SPEC §8b layout; the per-byte case below covers any other offset)
      const bool buy4 = (p.o_buy & 3) == 0;
      if (buy4) {
        uint32_t* b32 = reinterpret_cast<uint32_t*>(mb + p.o_buy);
        for (int j4 = lane; j4 < NMMO_MARKET_ROWS / 4; j4 += 64) {
          uint32_t v = 0u;
          if (exch && 4 * j4 < nm) {
            const uint2 q = *reinterpret_cast<const uint2*>(mpo + 4 * j4);
#pragma unroll
            for (int b = 0; b < 4; b++) {
              const uint32_t pw = ((b < 2 ? q.x : q.y) >> (16 * (b & 1))) & 0xFFFFu;
              if (4 * j4 + b < nm && (int)(pw & 255u) <= gold && (int)(pw >> 8) != a) v |= 1u << (8 * b);
            }
          }
          b32[j4] = v;
        }
        if (lane == 0) mb[p.o_buy + NMMO_MARKET_ROWS] = 1;
      }
      // one uniform loop over (section, 64-entry chunk): the section is a scalar, so its case runs
      // without divergence and only its own operands are live
      int sec = 0, k0 = 0;
#pragma unroll 1
      while (sec < 12) {
        int lo, n;
        switch (sec) {
          case 0: lo = p.o_style; n = p.o_target - p.o_style; break;
          case 1: lo = p.o_target; n = kNObs + 1; break;
          case 2: lo = p.o_buy; n = buy4 ? 0 : NMMO_MARKET_ROWS + 1; break;
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
        const int k = k0 + lane;
        if (k < n) {
          bool v;
          switch (sec) {
            case 0: v = combat; break;
            case 1:
              if (k == kNObs) {
                v = true;
              } else if (!combat || k >= nv) {
                v = false;
              } else {
                const int q = vis[k];
                v = q != a && linf(r, c, T[F_ROW * S + q], T[F_COL * S + q]) <= 3 &&
                    !(q < p.P && T[F_TIME_ALIVE * S + q] < p.spawn_immunity);
                if constexpr (kWrap)
                  if ((p.wflags & kWrapObsNoDangerous) && T[F_NPC_TYPE * S + q] > 1) v = false;
              }
              break;
            case 2:
              v = k == NMMO_MARKET_ROWS || (exch && k < nm && (int)(mpo[k] & 255u) <= gold && (int)(mpo[k] >> 8) != a);
              break;
            case 3: v = k == kInv || (item && free_item(k)); break;
            case 4: v = k == kInv || (!no_give && item && free_item(k)); break;
            case 5: v = k == kNObs || (!no_give && item && k < nv && same_tile(k)); break;
            case 6: v = exch && k < gold && (!no_give || k == 0); break;
            case 7: v = k == kNObs || (!no_give && exch && k < nv && same_tile(k)); break;
            case 8: v = !impassable(wmat[(kVision + dir_dr(k)) * 15 + kVision + dir_dc(k)]); break;
            case 9: v = k == kInv || (exch && k < ninv && !it_equipped(inv[k])); break;
            case 10:
              v = exch;
              if constexpr (kWrap)
                if ((p.wflags & kWrapObsPrice) && k == prev_price) v = false;
              break;
            default: v = k == kInv || (item && k < ninv && item_usable(T, S, a, inv[k])); break;
          }
          mb[lo + k] = v ? 1 : 0;
        }
        k0 += 64;
        if (k0 >= n) {
          sec++;
          k0 = 0;
        }
      }
      if (lane < NMMO_NATIVE_MASK_BYTES - p.o_agent_id) mb[p.o_agent_id + lane] = 0;
      // int16 part: AgentId, CurrentTick, Entity 100x31, Inventory 12x16, Tile 225x3, task index,
      // zero pads (SPEC §8b)
      int16_t* d16 = reinterpret_cast<int16_t*>(nrow + NMMO_NATIVE_MASK_BYTES);
      if (lane == 0) d16[0] = (int16_t)aid;
      if (lane == 1) d16[1] = (int16_t)tick;
      {  // two entity rows per pass: lanes 0-30 row k, lanes 32-62 row k + 1, one column each
        const int f = lane & 31, half = lane >> 5;
#pragma unroll 1
        for (int k0 = 0; k0 < kNObs; k0 += 2) {
          const int k = k0 + half;
          if (f < NMMO_N_ENTITY_COLS)
            d16[kNatEntity + k * NMMO_N_ENTITY_COLS + f] = k < nv ? T[f * S + vis[k]] : (int16_t)0;
        }
      }
      for (int j = lane; j < kInv * 16; j += 64) {
        const int k = j >> 4;
        d16[kNatInv + j] = k < ninv ? (int16_t)(int)item_col(inv[k], aid, j & 15) : (int16_t)0;
      }
#pragma unroll 1
      for (int i = 0; i < 4; i++) {
        const int t = lane + 64 * i;
        if (t < 225) {
          const int tr = r + t / 15 - kVision, tc = c + t % 15 - kVision;
          d16[kNatTile + 3 * t] = (int16_t)tr;
          d16[kNatTile + 3 * t + 1] = (int16_t)tc;
          d16[kNatTile + 3 * t + 2] = (int16_t)wm[i];
        }
      }
      if (lane == 0) d16[kNatTask] = (int16_t)p.assign[(size_t)e * p.P + a];
      else if (lane < NMMO_NATIVE_I16 - kNatTask) d16[kNatTask + lane] = 0;
      __builtin_amdgcn_wave_barrier();
      continue;
    }
    for (int j = lane; j < p.o_agent_id; j += 64) obs_st(&row[j], mask_val(j) ? 1.f : 0.f);
    if (lane == 0) obs_st(&row[p.o_agent_id], (float)aid);
    if (lane == 1) obs_st(&row[p.o_tick], (float)tick);
    // Entity rows (31 columns each)
    const int ne = kNObs * NMMO_N_ENTITY_COLS;
    for (int j = lane; j < ne; j += 64) {
      const int k = j / NMMO_N_ENTITY_COLS, f = j - k * NMMO_N_ENTITY_COLS;
      obs_st(&row[p.o_entity + j], k < nv ? (float)T[f * S + vis[k]] : 0.f);
    }
    // Inventory (own items, owner = self) and Market (env listings, ascending row)
    for (int j = lane; j < kInv * 16; j += 64) {
      const int k = j >> 4;
      obs_st(&row[p.o_inventory + j], k < ninv ? item_col(inv[k], aid, j & 15) : 0.f);
    }
    for (int j = lane; j < nm * 16; j += 64)
      obs_st(&row[p.o_market + j], item_col(mitem[j >> 4], mown[j >> 4] + 1, j & 15));
    wave_zero(row, p.o_market + nm * 16, p.o_task);
    const float* temb = p.task + (size_t)p.assign[(size_t)e * p.P + a] * p.task_dim;  // this player's task
    for (int j = lane; j < p.task_dim; j += 64) obs_st(&row[p.o_task + j], temb[j]);
    for (int j = lane; j < 225 * 3; j += 64) {
      const int t = j / 3, comp = j - 3 * t;
      const int tr = r + t / 15 - kVision, tc = c + t % 15 - kVision;
      obs_st(&row[p.o_tile + j], comp == 0 ? (float)tr : comp == 1 ? (float)tc : (float)mat[tr * kSize + tc]);
    }
    __builtin_amdgcn_wave_barrier();
  }
}

hipError_t launch_obs(const ObsParams& p, hipStream_t stream) {
  dim3 grid(p.n_envs, (p.P + kObsAgentsPerBlock - 1) / kObsAgentsPerBlock);
  const dim3 block(64 * kObsWaves);
  const size_t lds = obs_lds_bytes(p.S, p.nat != nullptr);
  if (p.nat) {
    if (p.wflags) hipLaunchKernelGGL((obs_kernel<true, true>), grid, block, lds, stream, p);
    else hipLaunchKernelGGL((obs_kernel<false, true>), grid, block, lds, stream, p);
  } else {
    if (p.wflags) hipLaunchKernelGGL((obs_kernel<true, false>), grid, block, lds, stream, p);
    else hipLaunchKernelGGL((obs_kernel<false, false>), grid, block, lds, stream, p);
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

__global__ void __launch_bounds__(512) policy_kernel(PolicyParams p) {
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

hipError_t launch_policy(const PolicyParams& p, hipStream_t stream) {
  if (p.S > 511) return hipErrorInvalidValue;  // grid entries hold ds_row - 1 in 9 bits
  hipLaunchKernelGGL(policy_kernel, dim3(p.n_envs), dim3(policy_threads(p.S, p.P)),
                     policy_lds_bytes(p.S, p.P), stream, p);
  return hipGetLastError();
}

}  // namespace nmmo
