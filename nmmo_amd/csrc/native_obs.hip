// native_obs.hip — NMMO_OBS_NATIVE: the per-agent observation gather in the nmmo-dtype layout
// of SPEC.md §8b (9,552 B per agent + the env's 32 KB Market), for learners that keep nmmo's
// dtypes (the flat float32 rows are nmmo_expand_obs of it, bit-identical).
//
// Staging, window compaction and the ActionTargets bit fields are agent_obs.h's (shared with
// the wire kernel). Per agent wave: the 1,586 u8 ActionTargets come from one 1,600-bit image
// held one dword per lane (the 11 uniform sections OR-ed into their lanes, Buy.MarketItem's 32
// entries per lane from the env's listings staged as price | owner << 8), expanded 16 bits ->
// 16 bytes per lane (two multiply-masks per dword) into 100 16-B stores; the int16 part goes out
// as dword stores (Entity row pairs are 31 dwords; Inventory 96 dwords; Tile + task index + pad
// 341 dwords) and one 16-B zero run for the unseen Entity rows. The workgroup's window rows and
// item words are staged in LDS up front (agent_obs.h ao_stage_windows), so the agent loop issues
// stores only and never waits on them.
#include "agent_obs.h"

namespace nmmo {

// The native kernel's workgroup: 32 agents on 8 waves (4 per wave, as agent_obs.h's 16 on 4), so
// the env's staged columns serve twice the rows per workgroup (round 6, same box: C4-native
// 359 -> 363 M, the kernel alone 0.093 -> 0.096 ms but overlapping the other batch's tick better;
// the flat and wire kernels measured slower with it and keep 16 on 4)
#ifndef NMMO_NO_WAVES  // (A/B knob: tools/debug/variants.py)
#define NMMO_NO_WAVES 8
#define NMMO_NO_AGENTS 32
#endif
constexpr int kNoWaves = NMMO_NO_WAVES, kNoAgents = NMMO_NO_AGENTS;
static_assert(kNoAgents / kNoWaves == kAoAgents / kAoWaves, "agents per wave: agent_obs.h's lane layouts");

// LDS: agent_obs.h's entity staging | listings (price | owner << 8, u16) | per-wave visible rows
// | the workgroup's staged window rows and item words. ~44 KB at S = 384 with 32 agents.
__host__ __device__ inline size_t no_lds_bytes(int S) {
  return ao_entity_lds(S) + (size_t)NMMO_MARKET_ROWS * 2 + (size_t)kNoWaves * 128 * 4 + ao_win_lds(kNoAgents);
}
constexpr int kNoEntity = 2, kNoInv = kNoEntity + kNObs * NMMO_N_ENTITY_COLS, kNoTile = kNoInv + kInv * 16,
              kNoTask = kNoTile + 225 * 3;  // int16 offsets in the int16 part (SPEC §8b)
static_assert(kNoTask < NMMO_NATIVE_I16 && (kNoTile & 1) == 0 && (NMMO_NATIVE_I16 & 1) == 0 &&
                  NMMO_NATIVE_MASK_BYTES % 16 == 0 && NMMO_NATIVE_ROW_BYTES % 16 == 0,
              "native layout");
constexpr int kNoImgWords = NMMO_NATIVE_MASK_BYTES / 32;  // 50: the mask image, one dword per lane

// (Capped at 96 VGPRs for a fifth wave per SIMD it measured 0.155 ms per 512 envs against 0.143
// uncapped at 109 VGPRs / 4 waves.)
template <bool kWrap>
__global__ void __launch_bounds__(64 * kNoWaves) native_obs_kernel(ObsParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int S = p.S, P = p.P, Sp = ao_stride(S);
  int16_t* T = reinterpret_cast<int16_t*>(smem);
  uint32_t* pk = reinterpret_cast<uint32_t*>(smem + ao_entity_lds(S) - (size_t)(kMaxSlots + 64) * 4);
  uint16_t* mpo = reinterpret_cast<uint16_t*>(pk + kMaxSlots + 64);           // [1024] price | owner << 8
  uint32_t* visw_all = reinterpret_cast<uint32_t*>(mpo + NMMO_MARKET_ROWS);   // [4][128]
  uint32_t* wst = visw_all + kNoWaves * 128;                                  // [16][15][5] window rows
  uint2* ist = reinterpret_cast<uint2*>(wst + kNoAgents * kAoWinAgentBytes / 4);  // [16][12] item words
#ifdef NMMO_NO_XCD  // 1-D grid, an env's groups back to back on one XCD (agent_obs.h ao_env_group)
  int el, g;
  ao_env_group(p.env_list ? p.n_list : p.n_envs, (p.P + kNoAgents - 1) / kNoAgents, el, g);
#else
  const int el = blockIdx.x, g = blockIdx.y;
#endif
  const int e = p.env_list ? p.env_list[el] : el, tid = threadIdx.x, lane = lane_id();
  if ((unsigned)e >= (unsigned)p.n_envs) return;  // a bad list id (the tick records it)
  const int w = __builtin_amdgcn_readfirstlane(wave_id());
  // the prologue in two memory round trips (as flat_obs.hip): the stage's loads with the
  // listings' count / mlist words and this wave's agents' words, then the listed items with the
  // windows
  AoStage sg;
  ao_stage_load(p, e, sg);
  const int16_t* E = p.ent + (size_t)e * NMMO_NF * S;
  const int per_wave = (kNoAgents + kNoWaves - 1) / kNoWaves;
  const int abase = g * kNoAgents + w;
  int my_task = 0, my_prev = -1, my_alive = 0;  // lane j: agent abase + 4 j
  uint64_t my_z = 0, my_s = 0;                  // its row state tag and word (ObsParams::zrow / zst)
  const bool mine = lane < per_wave && abase + kNoWaves * lane < P;
  {  // every lane loads (a clamped agent), the values kept for its own agent below
    const int aj = min(abase + kNoWaves * min(lane, per_wave - 1), P - 1);
    const size_t ai = (size_t)e * P + aj;
    my_task = p.assign[ai];
    my_alive = E[F_ALIVE * S + aj];
    if (p.ztag) {
      my_z = p.zrow[ai];
      my_s = p.zst[ai];
    }
    if constexpr (kWrap)
      if (p.ws) my_prev = p.ws[ai].prev_price;
  }
  ao_stage_store(p, e, T, pk, sg);
  if (!mine) {
    my_task = 0, my_prev = -1, my_alive = 0;
    my_z = my_s = 0;
  }
  const int nm = min(max(sg.nm, 0), NMMO_MARKET_ROWS);
  if (p.wmcount && g == 0 && tid == 0) p.wmcount[e] = nm;  // nmmo_wire_pack reads this launch's count
  const uint2 lwd = ao_listing_load(p, e, sg);
  ao_stage_windows<kNoAgents>(p, e, g, T, Sp, wst, ist, [&]() {  // the listings, ascending row (published by its barrier)
    if (tid < nm) mpo[tid] = (uint16_t)(it_price(lwd) | ((sg.mv >> 16) & 255) << 8);
    for (int j = tid + (int)blockDim.x; j < nm; j += blockDim.x) {  // (more listings than threads)
      const int v = p.mlist[(size_t)e * NMMO_MARKET_ROWS + j];
      const int own = (v >> 16) & 255, slot = (v >> 24) & 15;
      mpo[j] = (uint16_t)(it_price(p.items[((size_t)e * P + own) * kInv + slot]) | own << 8);
    }
  });

  uint8_t* nenv = p.nat + (size_t)e * ((size_t)P * NMMO_NATIVE_ROW_BYTES + NMMO_NATIVE_MARKET_BYTES);
  if (g == 0) {  // the env's Market (1,024 rows of 16 int16), once per env
    uint4* mk = reinterpret_cast<uint4*>(nenv + (size_t)P * NMMO_NATIVE_ROW_BYTES);
    for (int k = tid; k < NMMO_MARKET_ROWS; k += blockDim.x) {
      uint32_t q[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
      if (k < nm) {
        const int v = p.mlist[(size_t)e * NMMO_MARKET_ROWS + k];
        const int own = (v >> 16) & 255, slot = (v >> 24) & 15;
        const uint2 wd = p.items[((size_t)e * P + own) * kInv + slot];
#pragma unroll
        for (int i = 0; i < 8; i++)
          q[i] = i16pack((int)item_col(wd, own + 1, 2 * i), (int)item_col(wd, own + 1, 2 * i + 1));
      }
      mk[2 * k] = make_uint4(q[0], q[1], q[2], q[3]);
      mk[2 * k + 1] = make_uint4(q[4], q[5], q[6], q[7]);
    }
  }

  uint32_t pr[kAoRows];  // this lane's datastore rows 1 + lane + 64 i
#pragma unroll
  for (int i = 0; i < kAoRows; i++) pr[i] = pk[lane + 64 * i];
  uint32_t* visw = visw_all + w * 128;
  const uint8_t* wsb = reinterpret_cast<const uint8_t*>(wst);
  const int tick = p.env[(size_t)e * NMMO_NE + E_TICK];
  const bool exch = (p.systems & NMMO_SYS_ITEM) && (p.systems & NMMO_SYS_EXCHANGE);
  // bit j: agent j's row state describes this buffer / the row is all-zero already; my_h: the
  // Entity rows past which the row is zero (all 100 unknown, 0 for an all-zero row)
  const bool zvl = p.ztag && my_z == p.ztag;
  const uint64_t zvalid = __ballot(zvl), zknown = __ballot(zvl && (my_s & kZsZero));
  const int my_h = !zvl ? kNObs : (my_s & kZsZero) ? 0 : zs_hv(my_s);
  int nrows = 0;                  // rows this wave wrote (rows_out[0])
  unsigned long long nbytes = 0;  // bytes this wave stored (rows_out[1])
  int wo[2];
  ao_win_offsets(wo);
  auto alive = [&](int j) { return j < per_wave && __builtin_amdgcn_readlane(my_alive, j) != 0; };
  int toff[4];  // window tile lane + 64 i: (row offset) & 255 | (col offset) << 8
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int t = lane + 64 * i;
    toff[i] = ((t / 15 - kVision) & 255) | (t % 15 - kVision) * 256;
  }

  for (int j = 0; j < per_wave; j++) {
    const int a = abase + kNoWaves * j;
    if (a >= P) break;
    uint8_t* nrow = nenv + (size_t)a * NMMO_NATIVE_ROW_BYTES;
    if (!alive(j)) {  // not in the realm: a zero row
      if (p.wcount && lane == 0) p.wcount[(size_t)e * P + a] = 0;
      if ((zknown >> j) & 1) continue;  // zeroed by an earlier launch into this buffer
      uint4* z = reinterpret_cast<uint4*>(nrow);
      for (int i = lane; i < NMMO_NATIVE_ROW_BYTES / 16; i += 64) z[i] = make_uint4(0u, 0u, 0u, 0u);
      if (p.ztag && lane == 0) {
        p.zrow[(size_t)e * P + a] = p.ztag;
        p.zst[(size_t)e * P + a] = kZsZero;
      }
      nrows++;
      nbytes += NMMO_NATIVE_ROW_BYTES;
      continue;
    }
    nrows++;
    const int hv = __builtin_amdgcn_readlane(my_h, j);
    const int r = __builtin_amdgcn_readfirstlane(T[F_ROW * Sp + a]);
    const int c = __builtin_amdgcn_readfirstlane(T[F_COL * Sp + a]);
    const int gold = __builtin_amdgcn_readfirstlane(T[F_GOLD * Sp + a]);
    const int aid = __builtin_amdgcn_readfirstlane(T[F_ID * Sp + a]);
    // window tile t = lane + 64 i and item word lane, from the workgroup's staging
    const uint8_t* wa = wsb + (a - g * kNoAgents) * kAoWinAgentBytes + ((c - kVision) & 3);
    uint32_t wm[4];
#pragma unroll
    for (int i = 0; i < 4; i++) wm[i] = lane + 64 * i < 225 ? wa[ao_win_off(wo, i)] : 0u;
    const uint2 it = lane < kInv ? ist[(a - g * kNoAgents) * kInv + lane] : make_uint2(0u, 0u);
    const uint32_t mv = ao_move_bits(wm[1]);
    const int ninv = __builtin_ctzll(~__ballot(lane < kInv && it_type(it) != 0));  // occupied prefix

    const int nv = min(ao_compact(pr, S, r, c, visw), kNObs);
    if (p.wcount && lane == 0) p.wcount[(size_t)e * P + a] = (uint16_t)wire_count_word(nv, ninv);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    // ActionTargets: the 1,600-bit flat image, dword d in lane d
    {
      AoAgent ag;
      ag.a = a;
      ag.ti = a;
      ag.r = r;
      ag.c = c;
      ag.gold = gold;
      ag.aid = aid;
      ag.nv = nv;
      ag.ninv = ninv;
      ag.prev_price = kWrap ? __builtin_amdgcn_readlane(my_prev, j) : -1;
      ag.mv = mv;
      uint32_t img[kNoImgWords];
      ao_image<true>(ao_sections<kWrap>(p, T, Sp, visw, ag, it), img);
      img[(kWireBuyLo + NMMO_MARKET_ROWS) / 32] |= 1u << ((kWireBuyLo + NMMO_MARKET_ROWS) & 31);  // Buy noop
      // the section words (dwords 0-3 and 35-49: Buy.MarketItem fills the ones between)
      static_assert(sec_flat(2) / 32 == 3 && (sec_flat(3) - 1) / 32 == 35, "Buy.MarketItem dwords");
      int x = 0;
      x = writelanes<0, 0, 4>(img, x);
      x = writelanes<35, 35, kNoImgWords - 35>(img, x);
      // Buy.MarketItem entry k < listings (a lane per listing, 64 per ballot): exchange on,
      // price <= gold, not the agent's own; the ballot of listings j0 .. j0 + 63 covers flat bits
      // 104 + j0 .. (dwords 3 + j0 / 32 .. + 2, shifted by 8)
      if (exch) {
        for (int j0 = 0; j0 < nm; j0 += 64) {
          const int k = j0 + lane;
          bool bv = false;
          if (k < nm) {
            const uint32_t po = mpo[k];
            bv = (int)(po & 255u) <= gold && (int)(po >> 8) != a;
          }
          const uint64_t b = __ballot(bv);
          const int d0 = (kWireBuyLo + j0) >> 5;
          static_assert((kWireBuyLo & 31) == 8, "Buy.MarketItem bit shift");
          const uint32_t p0 = (uint32_t)(b << 8), p1 = (uint32_t)(b >> 24), p2 = (uint32_t)(b >> 56);
          x |= (int)(lane == d0 ? p0 : lane == d0 + 1 ? p1 : lane == d0 + 2 ? p2 : 0u);
        }
      }
      // 16 entries per lane -> 16 bytes: entry b of a nibble n lands in byte b by n * 0x204081
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const int q = 64 * h + lane;  // 16-B chunk
        const uint32_t b16 = ((uint32_t)__shfl(x, q >> 1) >> (16 * (q & 1))) & 0xFFFFu;
        if (q < NMMO_NATIVE_MASK_BYTES / 16) {
          uint32_t o[4];
#pragma unroll
          for (int i = 0; i < 4; i++) o[i] = (((b16 >> (4 * i)) & 15u) * 0x00204081u) & 0x01010101u;
          reinterpret_cast<uint4*>(nrow)[q] = make_uint4(o[0], o[1], o[2], o[3]);
        }
      }
    }
    // int16 part: AgentId, CurrentTick | Entity 100 x 31 | Inventory 12 x 16 | Tile 225 x 3 | task
    // index | zero pad (SPEC §8b)
    uint32_t* d32 = reinterpret_cast<uint32_t*>(nrow + NMMO_NATIVE_MASK_BYTES);
    if (lane == 0) d32[0] = i16pack(aid, tick);
    {  // four Entity rows per pass: a row pair is 31 dwords, lanes 0-30 the pair (k, k + 1), lanes
       // 32-62 the pair (k + 2, k + 3); the rows past the visible ones (rounded up to the pass)
       // are one zero run
      const int i = lane & 31, hp = lane >> 5;
      const int c0 = 2 * i, c1 = 2 * i + 1;
      const int r0 = c0 >= NMMO_N_ENTITY_COLS, r1 = c1 >= NMMO_N_ENTITY_COLS;
      const int f0 = c0 - r0 * NMMO_N_ENTITY_COLS, f1 = c1 - r1 * NMMO_N_ENTITY_COLS;
      const int nv4 = (nv + 3) & ~3;
      const int hz = max(nv4, hv);  // the rows past the visible ones not known zero
      uint32_t* de = d32 + kNoEntity / 2;
#pragma unroll 1
      for (int k0 = 0; k0 < nv4; k0 += 4) {
        const int k = k0 + 2 * hp, ka = k + r0, kb = k + r1;
        if (i < NMMO_N_ENTITY_COLS) {
          const int lo = ka < nv ? T[f0 * Sp + ao_slot(visw[ka])] : 0;
          const int hi = kb < nv ? T[f1 * Sp + ao_slot(visw[kb])] : 0;
          de[(k >> 1) * NMMO_N_ENTITY_COLS + i] = i16pack(lo, hi);
        }
      }
      uint8_t* zb = nrow + NMMO_NATIVE_MASK_BYTES + 2 * (kNoEntity + nv4 * NMMO_N_ENTITY_COLS);
      uint8_t* ze = nrow + NMMO_NATIVE_MASK_BYTES + 2 * (kNoEntity + hz * NMMO_N_ENTITY_COLS);
      nbytes += NMMO_NATIVE_ROW_BYTES - 2 * (kNObs - hz) * NMMO_N_ENTITY_COLS;
      if (p.ztag && lane == 0) {
        if (!((zvalid >> j) & 1)) p.zrow[(size_t)e * P + a] = p.ztag;
        p.zst[(size_t)e * P + a] = zs_pack(nv4, 0, 0);
      }
      // [zb, ze): 4-B aligned; dwords up to 16-B alignment, then 16-B stores, then dwords
      const int nz = (int)(ze - zb) >> 2;
      const int head = min((int)(((16 - (reinterpret_cast<uintptr_t>(zb) & 15)) & 15) >> 2), nz);
      if (lane < head) reinterpret_cast<uint32_t*>(zb)[lane] = 0u;
      const int body = (nz - head) >> 2;
      uint4* z4 = reinterpret_cast<uint4*>(zb + 4 * head);
      for (int q = lane; q < body; q += 64) z4[q] = make_uint4(0u, 0u, 0u, 0u);
      const int t0 = head + 4 * body;
      if (t0 + lane < nz) reinterpret_cast<uint32_t*>(zb)[t0 + lane] = 0u;
    }
    // Inventory: 96 dwords (item q = i >> 3, columns 2i & 15, +1), the item word from lane q
    if (ninv == 0) {
      if (lane < kInv * 8 / 4) reinterpret_cast<uint4*>(d32 + kNoInv / 2)[lane] = make_uint4(0u, 0u, 0u, 0u);
    } else {
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const int i = 64 * h + lane;
        const int q = min(i >> 3, kInv - 1);
        const uint2 iw = make_uint2((uint32_t)__shfl((int)it.x, q), (uint32_t)__shfl((int)it.y, q));
        if (i < kInv * 8) {
          const int cc = (2 * i) & 15;
          d32[kNoInv / 2 + i] =
              (i >> 3) < ninv ? i16pack((int)item_col(iw, aid, cc), (int)item_col(iw, aid, cc + 1)) : 0u;
        }
      }
    }
    // Tile: (row, col, material) per window tile t = lane + 64 i as three int16 stores (the
    // lane's row / column offsets are per-wave constants), then the task index and the zero pad
    {
      int16_t* d16 = reinterpret_cast<int16_t*>(d32) + kNoTile;
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int t = lane + 64 * i;
        if (t < 225) {
          d16[3 * t] = (int16_t)(r + ((toff[i] << 24) >> 24));
          d16[3 * t + 1] = (int16_t)(c + (toff[i] >> 8));
          d16[3 * t + 2] = (int16_t)wm[i];
        }
      }
      if (lane < NMMO_NATIVE_I16 - kNoTask)
        d16[225 * 3 + lane] = lane == 0 ? (int16_t)__builtin_amdgcn_readlane(my_task, j) : (int16_t)0;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the next agent reuses visw
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  if (p.rows_out && lane == 0 && nrows) {  // per env: one address per env keeps the atomics uncontended
    atomicAdd(&p.rows_out[2 * e], (unsigned long long)nrows);
    atomicAdd(&p.rows_out[2 * e + 1], nbytes);
  }
}

hipError_t launch_native_obs(const ObsParams& p, hipStream_t stream) {
  if (p.S % 8 || p.S > kMaxSlots || p.P > 128 || !p.nat || !ao_layout_ok(p)) return hipErrorInvalidValue;
  const int ne = list_grid(p.env_list, p.n_list, p.n_envs);
  if (ne <= 0) return hipSuccess;
#ifdef NMMO_NO_XCD
  const dim3 grid(ne * ((p.P + kNoAgents - 1) / kNoAgents)), block(64 * kNoWaves);
#else
  const dim3 grid(ne, (p.P + kNoAgents - 1) / kNoAgents), block(64 * kNoWaves);
#endif
  const size_t lds = no_lds_bytes(p.S);
  if (p.wflags) hipLaunchKernelGGL(native_obs_kernel<true>, grid, block, lds, stream, p);
  else hipLaunchKernelGGL(native_obs_kernel<false>, grid, block, lds, stream, p);
  return hipGetLastError();
}

}  // namespace nmmo
