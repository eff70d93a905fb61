// flat_obs.hip — the pufferlib-flat float32 obs rows (23,987 per agent, SPEC.md §8) written
// incrementally into the handle's bound buffer (nmmo_obs_bind): a row stores only
// what differs from what the buffer already holds (ObsParams::zrow / zst). Replaces
// Env._compute_observations + pufferlib's flatten/pad (the rows the reference's learner decodes with
// unpack_batched_obs, baseline_policy.py:41) for the bound buffer; an unbound or untracked buffer
// gets every row in full from obs.hip's obs_kernel<kWrap, true>.
//
// Round 5 rewrite on agent_obs.h's pieces (the native kernel's staging, compaction and section bit
// fields). The round-4 flat kernel was issue-bound (per agent row 760 VALU, 524 SALU, 146 branch
// for 33 stores; profiles/r04/pmc_flat): one predicate per mask entry, index arithmetic per store,
// 31-way LDS bank conflicts on the Entity gathers and SGPR spills. Here, per agent wave:
//  - ActionTargets: 25 chunks of 64 entries; chunk c's 64-bit mask is the OR of the sections' bit
//    fields at compile-time shifts (the Buy.MarketItem part from one ballot per 64 listings), and
//    lane L stores bit L of it as 0.f / 1.f -- one v_cndmask on the SGPR pair
//    (__builtin_amdgcn_inverse_ballot_w64) and one store per chunk. Chunks holding only Buy entries
//    at or past the row's known-zero threshold are skipped. AgentId / CurrentTick ride in the last
//    chunk's lanes 50 and 51;
//  - the env's Entity columns staged with an odd dword stride (conflict-free lane-per-field reads),
//    the window compaction from packed datastore-row words held in registers, and the workgroup's
//    window rows and item words staged in LDS up front, so the agent loop issues no global load
//    (except a Task section to rewrite, once per task change, and listings past the staged 256);
//  - every store goes to the row's wave-uniform base (SGPRs) plus a per-lane constant offset.
#include "agent_obs.h"

namespace nmmo {

#ifndef NMMO_FO_ABL  // diagnostic ablation (timing attribution only, wrong rows): bit 1 masks, 2 Entity,
#define NMMO_FO_ABL 0  // 4 Inventory, 8 Market, 16 Tile, 32 compaction, 64 the agent loop (prologue only),
#endif                 // 128 everything (an empty launch), 256 rows aliased onto 128 per XCD (stores L2-resident)
                       // (tools/debug/variants.py)
#ifndef NMMO_FO_STAMPS  // diagnostic: s_memtime per section of every alive row (tools/debug/fo_stamps.py)
#define NMMO_FO_STAMPS 0
#endif
#if NMMO_FO_STAMPS
constexpr int kFoStamps = 12;  // loop top, compaction, sections, chunks 0-1, Buy-only chunks, tail chunks,
                              // Entity, Inventory, Market, Task, Tile, state
__device__ uint64_t fo_stamp_buf[1 << 17][kFoStamps];
__device__ uint64_t fo_wave_buf[1 << 15][6];  // per wave: entry, staged, windows, loop start, loop end, env
#define FO_STAMP(k) fst[k] = __builtin_amdgcn_s_memtime()
#else
#define FO_STAMP(k) (void)0
#endif
#ifndef NMMO_FO_XCD  // (A/B knob: 1 = a 1-D grid with an env's groups on one XCD, agent_obs.h ao_env_group)
#define NMMO_FO_XCD 1
#endif
#ifndef NMMO_FO_TILE_SKIP  // (A/B knob: 1 = round 5's Tile component skip, tools/debug/variants.py)
#define NMMO_FO_TILE_SKIP 0
#endif
#ifndef NMMO_FO_TASK_BATCH  // (A/B knob: tools/debug/variants.py)
#define NMMO_FO_TASK_BATCH 8
#endif
constexpr int kFoTaskBatch = NMMO_FO_TASK_BATCH;  // Task floats per lane loaded before their stores
constexpr int kFoStagedListings = 256;  // listings whose item words are staged (Market rows)
constexpr int kFoChunks = 25;           // 64-entry chunks over the 1,586 mask entries (+ id, tick)
static_assert(kFoChunks * 64 >= kMaskN + 2 && (kFoChunks - 1) * 64 < kMaskN, "mask chunks");
static_assert(sec_flat(2) == 104 && sec_flat(3) == 104 + NMMO_MARKET_ROWS + 1, "Buy.MarketItem bits");
constexpr int kFoBuyLo = sec_flat(2);
// the flat row's section offsets (nmmo_layout; launch_flat_obs checks the handle's): compile-time,
// so the agent loop keeps few uniform values live (every runtime offset was an SGPR the loop spilled)
constexpr int kFoId = kMaskN, kFoEntity = kFoId + 2, kFoInv = kFoEntity + kNObs * NMMO_N_ENTITY_COLS,
              kFoMarket = kFoInv + kInv * 16, kFoTask = kFoMarket + NMMO_MARKET_ROWS * 16;

// LDS: agent_obs.h's entity staging | listings (price | owner << 8, u16) | the first 256 listings'
// item words | per-wave visible rows | the workgroup's staged window rows and item words.
// 38.7 KB at S = 384: 4 workgroups per CU.
__host__ __device__ inline size_t fo_lds_bytes(int S) {
  return ao_entity_lds(S) + (size_t)NMMO_MARKET_ROWS * 2 + (size_t)kFoStagedListings * 8 +
         (size_t)kAoWaves * 128 * 4 + ao_win_lds();
}

// Low 64 bits of the 128-bit field (hi:lo) shifted left by kSh (right when negative): the part of a
// section whose bit 0 sits at chunk bit kSh.
template <int kSh>
__device__ __forceinline__ uint64_t fo_shift(uint64_t lo, uint64_t hi) {
  if constexpr (kSh >= 64) {
    return 0ull;
  } else if constexpr (kSh > 0) {
    return lo << kSh;
  } else if constexpr (kSh == 0) {
    return lo;
  } else if constexpr (-kSh < 64) {
    return (lo >> (-kSh)) | (hi << (64 + kSh));
  } else if constexpr (-kSh < 128) {
    return hi >> (-kSh - 64);
  } else {
    return 0ull;
  }
}
// Section k's contribution to chunk kC (entries 64 kC .. 64 kC + 63 of the flat mask part)
template <int kK, int kC>
__device__ __forceinline__ uint64_t fo_sec(uint64_t lo, uint64_t hi) {
  constexpr int off = sec_flat(kK), n = kSecN[kK];
  if constexpr (off >= 64 * kC + 64 || off + n <= 64 * kC) return 0ull;
  else return fo_shift<off - 64 * kC>(lo, hi);
}
// The 11 section fields (every section but Buy.MarketItem) in chunk kC
template <int kC>
__device__ __forceinline__ uint64_t fo_chunk(const AoSections& x) {
  return fo_sec<0, kC>(x.s0, 0ull) | fo_sec<1, kC>(x.s1[0], x.s1[1]) | fo_sec<3, kC>(x.s3, 0ull) |
         fo_sec<4, kC>(x.s4, 0ull) | fo_sec<5, kC>(x.s5[0], x.s5[1]) | fo_sec<6, kC>(x.s6[0], x.s6[1]) |
         fo_sec<7, kC>(x.s7[0], x.s7[1]) | fo_sec<8, kC>(x.s8, 0ull) | fo_sec<9, kC>(x.s9, 0ull) |
         fo_sec<10, kC>(x.s10[0], x.s10[1]) | fo_sec<11, kC>(x.s11, 0ull);
}
__device__ __forceinline__ float fo_bit(uint64_t m) { return __builtin_amdgcn_inverse_ballot_w64(m) ? 1.f : 0.f; }
// row[idx] = v as base + zero-extended 32-bit byte offset: the store's SGPR-base (saddr) form, one
// offset VGPR, instead of a sign-extended 64-bit address built per store (4 VALU each)
__device__ __forceinline__ void fo_st(float* row, uint32_t idx, float v) {
  *reinterpret_cast<float*>(reinterpret_cast<char*>(row) + (idx << 2)) = v;
}

// The row's tracked ActionTargets chunks (ObsParams::zext): chunks 0 and 1 (Style, Attack.Target,
// Buy's first 24 entries) and 17..24 (Buy's last 40 entries and no-op, then every other section,
// AgentId, CurrentTick) as slots 0..9. A chunk whose mask equals the one the row was last written
// with is not stored again: per tick an agent's Move and Attack.Target bits change, while the
// gold-, inventory- and same-tile-driven sections mostly do not.
constexpr int kFoTail0 = (kFoBuyLo + NMMO_MARKET_ROWS) / 64;  // 17
__host__ __device__ constexpr int fo_slot(int c) { return c < 2 ? c : c - kFoTail0 + 2; }
static_assert(fo_slot(kFoChunks - 1) == 9 && kZext == 10 + 1 + 12, "tracked chunks | position | items");
struct FoImg {
  bool ext;        // the row's extended state is valid (else every chunk is stored)
  uint32_t lo, hi; // the wave's loaded masks: lane 10 j + slot = agent j's chunk `slot`
  int j10;         // 10 j
  int nimg;        // the new masks: lane 2 slot / 2 slot + 1 = slot's lo / hi word
  int nst;         // mask entries (+ id, tick) stored
};
__device__ __forceinline__ uint64_t fo_prev(const FoImg& g, int slot) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)g.lo, g.j10 + slot) |
         (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)g.hi, g.j10 + slot) << 32;
}
// chunk kC with mask m: stored unless the row holds it already; its mask goes into the new image
template <int kC>
__device__ __forceinline__ void fo_put(float* row, FoImg& g, uint64_t m, float aid, float tick) {
  constexpr int sl = fo_slot(kC);
  const int lane = ao_lane();
  const bool same = g.ext && m == fo_prev(g, sl);
  if constexpr (kC == kFoChunks - 1) {  // + AgentId, CurrentTick right after the mask entries
    constexpr int n = kMaskN - 64 * kC;
    if (!same) {
      if (lane < n + 2) fo_st(row, 64 * kC + lane, lane < n ? fo_bit(m) : lane == n ? aid : tick);
      g.nst += n + 2;
    } else {
      if (lane == n + 1) fo_st(row, 64 * kC + lane, tick);  // the tick changes every step
      g.nst += 1;
    }
  } else if (!same) {
    fo_st(row, 64 * kC + lane, fo_bit(m));
    g.nst += 64;
  }
  g.nimg = writelane<2 * sl>((int)(uint32_t)m, g.nimg);
  g.nimg = writelane<2 * sl + 1>((int)(uint32_t)(m >> 32), g.nimg);
}
template <int kC>
__device__ __forceinline__ void fo_tail_chunks(float* row, FoImg& g, const AoSections& x, uint64_t buy17, float aid,
                                               float tick) {
  if constexpr (kC < kFoChunks) {
    uint64_t m = fo_chunk<kC>(x);
    if constexpr (kC == kFoTail0) m |= buy17 | 1ull << ((kFoBuyLo + NMMO_MARKET_ROWS) & 63);
    fo_put<kC>(row, g, m, aid, tick);
    fo_tail_chunks<kC + 1>(row, g, x, buy17, aid, tick);
  }
}

// item_col (common.h) for a column fixed per lane (Inventory / Market chunks: lane L holds
// column L % 16 of every item it writes): a per-lane descriptor built once, so an entry is one
// bit-field extract plus a type-mask term instead of a 16-way select per entry.
//   value = bfe(x or y, sh, wd) + own * owner + mult * level + (mult ? b : 0),
//   mult = bit(type) of tmA * aA + bit(type) of tmB * aB
struct IcDesc {
  uint32_t tmA, tmB;
  uint32_t f;  // sel | sh << 1 | wd << 6 | own << 11 | aA << 12 | aB << 16 | b << 20
};
__device__ __forceinline__ IcDesc ic_desc(int col) {
  auto bits = [](int lo, int hi) { return ((2u << hi) - 1u) & ~((1u << lo) - 1u); };
  IcDesc d{0u, 0u, 0u};
  auto bf = [&](int sel, int sh, int wd) { d.f = (uint32_t)(sel | sh << 1 | wd << 6); };
  switch (col) {
    case 0: bf(1, 16, 16); break;  // row
    case 1: bf(0, 0, 5); break;    // type
    case 2: d.f = 1u << 11; break; // owner
    case 3: bf(0, 5, 4); break;    // level
    case 5: bf(1, 0, 16); break;   // quantity
    case 6: case 7: case 8:        // melee / range / mage attack
      d.tmA = 1u << (T_SPEAR + col - 6) | 1u << (T_WHETSTONE + col - 6);
      d.f = 5u << 12 | 5u << 20;
      break;
    case 9: case 10: case 11:      // defense
      d.tmA = bits(T_HAT, T_BOTTOM);
      d.tmB = bits(T_ROD, T_CHISEL);
      d.f = 3u << 12 | 2u << 16;
      break;
    case 12: d.tmA = 1u << T_POTION; d.f = 5u << 12 | 50u << 20; break;
    case 13: d.tmA = 1u << T_RATION; d.f = 5u << 12 | 50u << 20; break;
    case 14: bf(0, 9, 1); break;   // equipped
    case 15: bf(0, 10, 7); break;  // listed price
    default: break;                // 4: zero
  }
  return d;
}
__device__ __forceinline__ float ic_value(uint2 w, int owner, const IcDesc& d) {
  const int type = (int)(w.x & 31u), lvl = (int)((w.x >> 5) & 15u);
  const uint32_t bfv = __builtin_amdgcn_ubfe((d.f & 1u) ? w.y : w.x, (d.f >> 1) & 31u, (d.f >> 6) & 31u);
  const int ta = (int)((d.tmA >> type) & 1u), tb = (int)((d.tmB >> type) & 1u);
  const int mult = ta * (int)((d.f >> 12) & 15u) + tb * (int)((d.f >> 16) & 15u);
  return (float)((int)bfv + (int)((d.f >> 11) & 1u) * owner + mult * lvl + ((ta | tb) ? (int)(d.f >> 20) : 0));
}
static_assert(T_POTION < 32 && T_RATION < 32 && T_WHETSTONE + 2 < 32, "item type masks");

// Window compaction as agent_obs.h's ao_compact over all kAoRows register words (the rows past S
// hold kAoEmpty, outside every window): no bound on S to keep live across the agent loop
__device__ __forceinline__ int fo_compact(const uint32_t (&pr)[kAoRows], int r, int c, uint32_t* visw) {
  int nvis = 0;
  const uint32_t rc = (uint32_t)r | (uint32_t)c << 16;
#pragma unroll
  for (int i = 0; i < kAoRows; i++) {
    const bool in = ao_in_window(pr[i], rc);
    const uint64_t b = __ballot(in);
    const int pos = nvis + __popcll(b & lanes_below());
    if (in && pos < kNObs) visw[pos] = pr[i];
    nvis += __popcll(b);
  }
  return nvis;
}

typedef const __attribute__((address_space(4))) ObsParams* FoArgs;  // the kernel's argument segment

// kS: the slot count when known at compile time (C3 / C4: 128 players + 256 NPCs), 0 = p.S. With
// it the staged-column offsets are immediates instead of uniform values the agent loop keeps live.
template <bool kWrap, int kS>
__global__ void __launch_bounds__(64 * kAoWaves) flat_obs_kernel(ObsParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int S = kS ? kS : p.S, P = p.P, Sp = ao_stride(S), tdim = p.task_dim, elems = kFoTask + tdim + 225 * 3;
  int16_t* T = reinterpret_cast<int16_t*>(smem);
  uint32_t* pk = reinterpret_cast<uint32_t*>(smem + ao_entity_lds(S) - (size_t)(kMaxSlots + 64) * 4);
  uint16_t* mpo = reinterpret_cast<uint16_t*>(pk + kMaxSlots + 64);            // [1024] price | owner << 8
  uint2* mitem = reinterpret_cast<uint2*>(mpo + NMMO_MARKET_ROWS);            // [256] listed item words
  uint32_t* visw_all = reinterpret_cast<uint32_t*>(mitem + kFoStagedListings);  // [4][128]
  uint32_t* wst = visw_all + kAoWaves * 128;                                   // [16][15][5] window rows
  uint2* ist = reinterpret_cast<uint2*>(wst + kAoAgents * kAoWinAgentBytes / 4);  // [16][12] item words
#if NMMO_FO_XCD  // 1-D grid, an env's groups back to back on one XCD (agent_obs.h ao_env_group)
  int el, g;
  ao_env_group(p.env_list ? p.n_list : p.n_envs, (p.P + kAoAgents - 1) / kAoAgents, el, g);
#else
  const int el = blockIdx.x, g = blockIdx.y;
#endif
  const int e = p.env_list ? p.env_list[el] : el, tid = threadIdx.x, lane = lane_id();
  if ((unsigned)e >= (unsigned)p.n_envs) return;  // a bad list id (the tick records it)
  if (NMMO_FO_ABL & 128) return;
#if NMMO_FO_STAMPS
  uint64_t wst_[6];
  wst_[0] = __builtin_amdgcn_s_memtime();
#endif
  const int w = __builtin_amdgcn_readfirstlane(wave_id());
  // The prologue in two memory round trips: (1) the stage's loads, the listings' count and mlist
  // words and this wave's agents' words; (2) after the stage's LDS writes, the listed items, the
  // agents' extended row state and the workgroup's windows. (Issued where each was first needed,
  // the count -> mlist -> item chain, the stage, the windows and the extended state were six.)
  AoStage sg;
  ao_stage_load(p, e, sg);
  const int16_t* E = p.ent + (size_t)e * NMMO_NF * S;
  constexpr int kPerWave = kAoAgents / kAoWaves;
  const int abase = g * kAoAgents + w;
  int my_task = 0, my_prev = -1, my_alive = 0;  // lane j: agent abase + 4 j
  uint64_t my_z = 0, my_s = 0;                  // its row state tag and word
  const bool mine = lane < kPerWave && abase + kAoWaves * lane < P;
  {  // every lane loads (a clamped agent), the values kept for its own agent below
    const int aj = min(abase + kAoWaves * min(lane, kPerWave - 1), P - 1);
    const size_t ai = (size_t)e * P + aj;
    my_task = p.assign[ai];
    my_alive = E[F_ALIVE * S + aj];
    if (p.zrow) {
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
#if NMMO_FO_STAMPS
  wst_[1] = __builtin_amdgcn_s_memtime();
#endif

  uint32_t pr[kAoRows];  // this lane's datastore rows 1 + lane + 64 i
#pragma unroll
  for (int i = 0; i < kAoRows; i++) pr[i] = pk[lane + 64 * i];
  uint32_t* visw = visw_all + w * 128;
  const uint8_t* wsb = reinterpret_cast<const uint8_t*>(wst);
  const float tickf = (float)p.env[(size_t)e * NMMO_NE + E_TICK];
  const bool exch = (p.systems & NMMO_SYS_ITEM) && (p.systems & NMMO_SYS_EXCHANGE);

  // bit j: agent j's row state describes this buffer / the row is all-zero / its Task section holds
  // its task's embedding / its extended state is valid; my_h = hv | hm << 12: its Entity rows >= hv
  // and its Market rows and Buy entries >= hm are zero (a row of unknown content: nothing known zero)
  const bool zvl = p.ztag && my_z == p.ztag;
  const bool zzl = zvl && (my_s & kZsZero);
  const uint64_t zvalid = __ballot(zvl), zzero = __ballot(zzl), ztask = __ballot(zvl && !zzl && zs_task(my_s) == my_task);
  const uint64_t zextv = __ballot(zvl && !zzl && (my_s & kZsExt));
  const uint64_t ztile = __ballot(zvl && (my_s & kZsTile));  // its Tile section was written by a consumer
  // the extended state (ObsParams::zext): lane 10 j + slot = agent j's tracked chunk `slot`, lane
  // 40 + j its Tile position; lane 12 j + k (inv) its item word k
  // (loaded by every lane from a valid address, with the listings' items and ahead of the
  // windows, and kept only where the state is valid)
  uint2 img = make_uint2(0u, 0u), pinv = make_uint2(0u, 0u);
  const int ja = lane < 40 ? lane / 10 : lane - 40, ji = lane / 12;
  const bool img_ok = lane < 44 && abase + kAoWaves * ja < P && ((zextv >> ja) & 1);
  const bool pinv_ok = lane < 48 && abase + kAoWaves * ji < P && ((zextv >> ji) & 1);
  if (p.zext) {
    const int aa = min(abase + kAoWaves * min(ja, kPerWave - 1), P - 1);
    const int ai = min(abase + kAoWaves * min(ji, kPerWave - 1), P - 1);
    img = reinterpret_cast<const uint2*>(p.zext)[((size_t)e * P + aa) * kZext + (lane < 40 ? lane % 10 : 10)];
    pinv = reinterpret_cast<const uint2*>(p.zext)[((size_t)e * P + ai) * kZext + 11 + min(lane, 47) % 12];
  }
  const int nm = min(max(sg.nm, 0), NMMO_MARKET_ROWS);
  const uint2 lwd = ao_listing_load(p, e, sg);
  // the listings (ascending row) into LDS ahead of the windows' barrier, which publishes them
  ao_stage_windows(p, e, g, T, Sp, wst, ist, [&]() {
    if (tid < nm) {
      mpo[tid] = (uint16_t)(it_price(lwd) | ((sg.mv >> 16) & 255) << 8);
      if (tid < kFoStagedListings) mitem[tid] = lwd;
    }
    for (int j = tid + (int)blockDim.x; j < nm; j += blockDim.x) {  // (more listings than threads)
      const int v = p.mlist[(size_t)e * NMMO_MARKET_ROWS + j];
      const int own = (v >> 16) & 255, slot = (v >> 24) & 15;
      const uint2 wd = p.items[((size_t)e * P + own) * kInv + slot];
      mpo[j] = (uint16_t)(it_price(wd) | own << 8);
      if (j < kFoStagedListings) mitem[j] = wd;
    }
  });
#if NMMO_FO_STAMPS
  wst_[2] = __builtin_amdgcn_s_memtime();
#endif
  // Every prologue load has been waited on (the windows' LDS writes): a first use of img / pinv /
  // my_prev inside the agent loop (under a branch the waitcnt pass cannot see through) waited for
  // every store the row had issued -- one full drain per tracked chunk.
  asm volatile("" : "+v"(img.x), "+v"(img.y), "+v"(pinv.x), "+v"(pinv.y), "+v"(my_prev));
  if (!img_ok) img = make_uint2(0u, 0u);
  if (!pinv_ok) pinv = make_uint2(0u, 0u);
  const int my_h = !zvl ? (kNObs | NMMO_MARKET_ROWS << 12) : zzl ? 0 : (zs_hv(my_s) | zs_hm(my_s) << 12);
  int nrows = 0;                  // rows this wave wrote (rows_out[0])
  unsigned long long nbytes = 0;  // bytes this wave stored (rows_out[1])
  int wo[2];
  ao_win_offsets(wo);
  int toff[4];  // window tile lane + 64 i: (row offset) & 255 | (col offset) << 8
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int t = lane + 64 * i;
    toff[i] = ((t / 15 - kVision) & 255) | (t % 15 - kVision) * 256;
  }
  const int ef = lane & 31, eh = lane >> 5;  // Entity: field, row of the pair
  const int iq = lane >> 4;                  // Inventory: item of the chunk
  const IcDesc icd = ic_desc(lane & 15);      // Inventory / Market: column lane % 16

#if NMMO_FO_STAMPS
  wst_[3] = __builtin_amdgcn_s_memtime();
#endif
#pragma unroll 1
  for (int j = 0; j < ((NMMO_FO_ABL & 64) ? 0 : kPerWave); j++) {
    const int a = abase + kAoWaves * j;
    if (a >= P) break;
    const int lane = ao_lane();  // (per iteration: lane predicates are not hoisted and spilled)
    // the kernel arguments the row's stores use, read from the argument segment per agent (scalar
    // loads) instead of held in SGPRs across the loop, which spilled them
    FoArgs kp = (FoArgs)__builtin_amdgcn_kernarg_segment_ptr();  // p is the only argument
    asm volatile("" : "+s"(kp));
    // the row pointer opaque per agent (its global address space kept), so the section bases are
    // computed from it in the loop instead of hoisted out of it (and spilled)
    auto grow = (__attribute__((address_space(1))) float*)(p.obs + ((NMMO_FO_ABL & 256)
        ? (size_t)(((e * P + a) & 15) + 16 * (blockIdx.x & 7)) : (size_t)e * P + a) * elems);
    asm volatile("" : "+s"(grow));
    float* row = (float*)grow;
    const bool zv = (zvalid >> j) & 1;
    const int hj = __builtin_amdgcn_readlane(my_h, j);
    const int hv = hj & 4095, hm = hj >> 12;
    if (!__builtin_amdgcn_readlane(my_alive, j)) {  // not in the realm: an all-zero row
      if ((zzero >> j) & 1) {  // zeroed by an earlier launch into this buffer
        if ((ztile >> j) & 1) {  // ... but a consumer wrote into its Tile section since
          wave_zero(row, kFoTask + tdim, elems);
          nbytes += 4ull * (elems - kFoTask - tdim);
          if (lane == 0) kp->zst[(size_t)e * P + a] = kZsZero;
          nrows++;
        }
        continue;
      }
      if (zv) {  // zero what the last write left nonzero
        wave_zero(row, 0, kFoEntity + hv * NMMO_N_ENTITY_COLS);
        wave_zero(row, kFoInv, kFoMarket + hm * 16);
        wave_zero(row, kFoTask, elems);
        nbytes += 4ull * (kFoEntity + hv * NMMO_N_ENTITY_COLS + kFoMarket + hm * 16 - kFoInv + elems - kFoTask);
      } else {
        wave_zero(row, 0, elems);
        nbytes += 4ull * elems;
      }
      if (lane == 0) {
        kp->zrow[(size_t)e * P + a] = kp->ztag;
        kp->zst[(size_t)e * P + a] = kZsZero;
      }
      nrows++;
      continue;
    }
    nrows++;
#if NMMO_FO_STAMPS
    uint64_t fst[kFoStamps];
#endif
    FO_STAMP(0);
    const int la = a - g * kAoAgents;
    const int r = __builtin_amdgcn_readfirstlane(T[F_ROW * Sp + a]);
    const int c = __builtin_amdgcn_readfirstlane(T[F_COL * Sp + a]);
    const int gold = __builtin_amdgcn_readfirstlane(T[F_GOLD * Sp + a]);
    const int aid = __builtin_amdgcn_readfirstlane(T[F_ID * Sp + a]);
    const uint8_t* wa = wsb + la * kAoWinAgentBytes + ((c - kVision) & 3);
    uint32_t wm[4];
#pragma unroll
    for (int i = 0; i < 4; i++) wm[i] = lane + 64 * i < 225 ? wa[ao_win_off(wo, i)] : 0u;
    const uint2 it = lane < kInv ? ist[la * kInv + lane] : make_uint2(0u, 0u);
    const uint32_t mv = ao_move_bits(wm[1]);
    const int ninv = __builtin_ctzll(~__ballot(lane < kInv && it_type(it) != 0));  // occupied prefix
    const int nv = (NMMO_FO_ABL & 32) ? 0 : min(fo_compact(pr, r, c, visw), kNObs);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    FO_STAMP(1);
    const bool ext = (zextv >> j) & 1;  // the row's extended state is valid
    FoImg fg{ext, img.x, img.y, 10 * j, 0, 0};
    // ActionTargets (+ AgentId, CurrentTick)
    if (!(NMMO_FO_ABL & 1)) {
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
      const AoSections x = ao_sections<kWrap>(p, T, Sp, visw, ag, it);
      FO_STAMP(2);
      fg.ext = ext;
      fo_put<0>(row, fg, fo_chunk<0>(x), 0.f, 0.f);
      // Buy.MarketItem entry k < listings: exchange on, price <= gold, not the agent's own. buy_word
      // m = the ballot over listings 64 m + lane; chunk c holds words c - 1 (from bit 40) and c - 2
      // (its top 40 bits). Chunks 2..16 hold Buy entries only: written up to the known-zero
      // threshold max(nm, hm) (their entries past nm are zero).
      auto buy_word = [&](int m) {
        const int k = 64 * m + lane;
        bool bv = false;
        if (exch && k < nm) {
          const uint32_t po = mpo[k];
          bv = (int)(po & 255u) <= gold && (int)(po >> 8) != a;
        }
        return __ballot(bv);
      };
      const int nbuy = max(nm, hm);
      const int clast = max(1, min((kFoBuyLo + nbuy - 1) >> 6, 16));
      uint64_t bprev = nm > 0 ? buy_word(0) : 0ull;  // chunk 1: Attack.Target's tail, Buy's first 24
      fo_put<1>(row, fg, fo_chunk<1>(x) | bprev << (kFoBuyLo & 63), 0.f, 0.f);
      FO_STAMP(3);
#pragma unroll 1
      for (int cc = 2; cc <= clast; cc++) {  // Buy-only chunks, not tracked
        const uint64_t bcur = 64 * (cc - 1) < nm ? buy_word(cc - 1) : 0ull;
        fo_st(row, 64 * cc + lane, fo_bit(bcur << (kFoBuyLo & 63) | bprev >> (64 - (kFoBuyLo & 63))));
        bprev = bcur;
      }
      // chunk 17: Buy entries 984..1023 (word 15, only when nm > 960: the loop then ran to 16)
      FO_STAMP(4);
      const uint64_t buy17 = nm > 15 * 64 ? bprev >> (64 - (kFoBuyLo & 63)) : 0ull;
      fo_tail_chunks<kFoTail0>(row, fg, x, buy17, (float)aid, tickf);
      nbytes += 4ull * (fg.nst + 64 * (clast - 1));
    }
    FO_STAMP(5);
    // Entity rows: two per pass (lanes 0-30 row k, lanes 32-62 row k + 1: 62 contiguous floats),
    // the rows past the visible ones not known zero as one zero run
    const int nv2 = (nv + 1) & ~1;
    if (!(NMMO_FO_ABL & 2)) {
      const uint32_t de = kFoEntity + (lane - eh);
#pragma unroll 1
      for (int k0 = 0; k0 < nv2; k0 += 2) {
        const int k = k0 + eh;
        if (ef < NMMO_N_ENTITY_COLS)
          fo_st(row, de + k0 * NMMO_N_ENTITY_COLS, k < nv ? (float)T[ef * Sp + ao_slot(visw[k])] : 0.f);
      }
      const int hz = max(nv2, hv);
      wave_zero(row, kFoEntity + nv2 * NMMO_N_ENTITY_COLS, kFoEntity + hz * NMMO_N_ENTITY_COLS);
      nbytes += 4ull * (hz * NMMO_N_ENTITY_COLS + max(nm, hm) * 16);
    }
    FO_STAMP(6);
    // Inventory: item q = 4 h + lane / 16, column lane % 16 (own items, owner = self); not stored
    // when the row was last written from the same 12 item words (its only inputs besides AgentId)
    const int jl = (12 * j + lane) & 63;
    const uint32_t px = (uint32_t)__shfl((int)pinv.x, jl), py = (uint32_t)__shfl((int)pinv.y, jl);
    const bool inv_same = ext && __ballot(lane < kInv && (px != it.x || py != it.y)) == 0ull;
    if (!inv_same) {
#pragma unroll
      for (int h = 0; h < ((NMMO_FO_ABL & 4) ? 0 : kInv * 16 / 64); h++) {
        const int q = 4 * h + iq;
        float v = 0.f;
        if (4 * h < ninv && q < ninv) v = ic_value(ist[la * kInv + q], aid, icd);  // (a uniform skip first)
        fo_st(row, kFoInv + 64 * h + lane, v);
      }
      nbytes += 4ull * kInv * 16;
    }
    FO_STAMP(7);
    // Market (the env's listings, ascending row; owner = lister) and its zero run down to hm
    // (the listings past the staged ones in a loop of their own: a global load in the common loop
    // made every iteration wait for all of the row's stores -- vmcnt counts stores and retires in
    // order -- whether or not it took the load)
    const int nms = (NMMO_FO_ABL & 8) ? 0 : min(nm, kFoStagedListings);
    for (int k = lane; k < nms * 16; k += 64) fo_st(row, kFoMarket + k, ic_value(mitem[k >> 4], (mpo[k >> 4] >> 8) + 1, icd));
    if (nm > nms && !(NMMO_FO_ABL & 8)) {
      for (int k = nms * 16 + lane; k < nm * 16; k += 64) {
        const int q = k >> 4;
        const int v = kp->mlist[(size_t)e * NMMO_MARKET_ROWS + q];
        const uint2 wd = kp->items[((size_t)e * P + ((v >> 16) & 255)) * kInv + ((v >> 24) & 15)];
        fo_st(row, kFoMarket + k, ic_value(wd, (mpo[q] >> 8) + 1, icd));
      }
    }
    wave_zero(row, kFoMarket + nm * 16, kFoMarket + max(nm, hm) * 16);
    FO_STAMP(8);
    // Task: only when the row does not hold this task's embedding yet (read in place)
    const int task = __builtin_amdgcn_readlane(my_task, j);
    if (!((ztask >> j) & 1)) {
      // kFoTaskBatch loads in flight before their stores: each load waits for every store issued
      // before it (vmcnt retires in order), so a load-store loop drained the queue per 64 floats
      const float* temb = kp->task + (size_t)task * tdim;
      int k0 = 0;
      for (; k0 + kFoTaskBatch * 64 <= tdim; k0 += kFoTaskBatch * 64) {
        float t[kFoTaskBatch];
#pragma unroll
        for (int i = 0; i < kFoTaskBatch; i++) t[i] = temb[k0 + 64 * i + lane];
#pragma unroll
        for (int i = 0; i < kFoTaskBatch; i++) fo_st(row, kFoTask + k0 + 64 * i + lane, t[i]);
      }
      for (int k = k0 + lane; k < tdim; k += 64) fo_st(row, kFoTask + k, temb[k]);
      nbytes += 4ull * tdim;
    }
    FO_STAMP(9);
    // Tile: (row, column, material) per window tile t = lane + 64 i, three stores 12 B apart, all
    // three every step: the three stores of a pass fill 768 contiguous bytes, so the section goes out
    // as whole lines. (Round 5 skipped the row / column components when the agent had not moved: a
    // third of the stores, but every line of the section was still written in part, which HBM writes
    // as whole sectors -- WRITE_SIZE 1.9x the stored bytes; NMMO_FO_TILE_SKIP=1 keeps that variant.)
    const uint32_t ppos = (uint32_t)__builtin_amdgcn_readlane((int)img.x, 40 + j);
    const bool tkn = NMMO_FO_TILE_SKIP && ext && !((ztile >> j) & 1);  // the Tile section holds what this kernel wrote
    const bool same_r = tkn && (int)(ppos & 255u) == r, same_c = tkn && (int)((ppos >> 8) & 255u) == c;
    if (!(NMMO_FO_ABL & 16)) {
      float* dt = row + kFoTask + tdim + 3 * lane;
#pragma unroll
      for (int i = 0; i < 4; i++) {
        if (lane + 64 * i < 225) {
          const float vr = (float)(r + ((toff[i] << 24) >> 24)), vc = (float)(c + (toff[i] >> 8)), vm = (float)wm[i];
          if (NMMO_FO_TILE_SKIP) {
            if (!same_r) dt[192 * i] = vr;
            if (!same_c) dt[192 * i + 1] = vc;
            dt[192 * i + 2] = vm;
          } else {  // the tile's 12 bytes as one 3-dword store (rows are 4-B aligned)
            typedef float f3 __attribute__((ext_vector_type(3)));
            const f3 v = {vr, vc, vm};
            __builtin_memcpy(dt + 192 * i, &v, 12);
          }
        }
      }
      nbytes += 4ull * 225 * (1 + !same_r + !same_c);
    }
    FO_STAMP(10);
    {  // the row's state: tag, zero thresholds and task, then the extended state
      uint32_t* zx = reinterpret_cast<uint32_t*>(kp->zext + ((size_t)e * P + a) * kZext);
      int wv = fg.nimg;  // lanes 0..19 the tracked masks, lanes 20 / 21 the position
      if (lane == 20) wv = r | c << 8;
      if (lane == 21) wv = 0;
      if (lane < 22) zx[lane] = (uint32_t)wv;
      if (!inv_same && lane < kInv) reinterpret_cast<uint2*>(zx + 22)[lane] = it;
      if (lane == 0) {
        if (!zv) kp->zrow[(size_t)e * P + a] = kp->ztag;
        kp->zst[(size_t)e * P + a] = zs_pack(nv2, nm, task) | kZsExt;
      }
    }
#if NMMO_FO_STAMPS
    FO_STAMP(11);
    if (lane == 0 && (size_t)e * P + a < (1u << 17))
      for (int k = 0; k < kFoStamps; k++) fo_stamp_buf[(size_t)e * P + a][k] = fst[k];
#endif
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the next agent reuses visw
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
#if NMMO_FO_STAMPS
  wst_[4] = __builtin_amdgcn_s_memtime();
  wst_[5] = (uint64_t)e | (uint64_t)nrows << 32;
  {
    const size_t wi = ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * kAoWaves + w;
    if (lane == 0 && wi < (1u << 15))
      for (int k = 0; k < 6; k++) fo_wave_buf[wi][k] = wst_[k];
  }
#endif
  if (p.rows_out && lane == 0 && nrows) {  // per env: one address per env keeps the atomics uncontended
    atomicAdd(&p.rows_out[2 * e], (unsigned long long)nrows);
    atomicAdd(&p.rows_out[2 * e + 1], nbytes);
  }
}

bool flat_obs_ok(const ObsParams& p) {  // agent_obs.h's staging: S a multiple of 8 (16-B column loads)
  return p.S % 8 == 0 && p.S <= kMaxSlots && p.P <= 128 && p.obs && p.ztag && p.zrow && ao_layout_ok(p) &&
         p.o_agent_id == kFoId && p.o_tick == kFoId + 1 && p.o_entity == kFoEntity && p.o_inventory == kFoInv &&
         p.o_market == kFoMarket && p.o_task == kFoTask && p.o_tile == kFoTask + p.task_dim &&
         p.elems == p.o_tile + 225 * 3;
}

hipError_t launch_flat_obs(const ObsParams& p, hipStream_t stream) {
  if (!flat_obs_ok(p)) return hipErrorInvalidValue;
  const int ne = list_grid(p.env_list, p.n_list, p.n_envs);
  if (ne <= 0) return hipSuccess;
#if NMMO_FO_XCD
  const dim3 grid(ne * ((p.P + kAoAgents - 1) / kAoAgents)), block(64 * kAoWaves);
#else
  const dim3 grid(ne, (p.P + kAoAgents - 1) / kAoAgents), block(64 * kAoWaves);
#endif
  const size_t lds = fo_lds_bytes(p.S);
  if (p.S == kMaxSlots) {
    if (p.wflags) hipLaunchKernelGGL((flat_obs_kernel<true, kMaxSlots>), grid, block, lds, stream, p);
    else hipLaunchKernelGGL((flat_obs_kernel<false, kMaxSlots>), grid, block, lds, stream, p);
  } else {
    if (p.wflags) hipLaunchKernelGGL((flat_obs_kernel<true, 0>), grid, block, lds, stream, p);
    else hipLaunchKernelGGL((flat_obs_kernel<false, 0>), grid, block, lds, stream, p);
  }
  return hipGetLastError();
}

}  // namespace nmmo

#if NMMO_FO_STAMPS
// diagnostic export of the stamp variant only: copy the stamps out, then zero them
extern "C" __attribute__((visibility("default"))) int nmmo_debug_fo_stamps(void* host, size_t bytes) {
  if (bytes > sizeof(nmmo::fo_stamp_buf)) bytes = sizeof(nmmo::fo_stamp_buf);
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(nmmo::fo_stamp_buf), bytes) != hipSuccess) return -1;
  void* d = nullptr;
  if (hipGetSymbolAddress(&d, HIP_SYMBOL(nmmo::fo_stamp_buf)) != hipSuccess) return -1;
  return hipMemset(d, 0, sizeof(nmmo::fo_stamp_buf)) == hipSuccess && hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}
extern "C" __attribute__((visibility("default"))) int nmmo_debug_fo_wave_stamps(void* host, size_t bytes) {
  if (bytes > sizeof(nmmo::fo_wave_buf)) bytes = sizeof(nmmo::fo_wave_buf);
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(nmmo::fo_wave_buf), bytes) != hipSuccess) return -1;
  void* d = nullptr;
  if (hipGetSymbolAddress(&d, HIP_SYMBOL(nmmo::fo_wave_buf)) != hipSuccess) return -1;
  return hipMemset(d, 0, sizeof(nmmo::fo_wave_buf)) == hipSuccess && hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}
#endif
