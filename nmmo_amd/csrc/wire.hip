// wire.hip — compact transport encoding of native observations (SPEC.md §8c) for the learner
// gather of BASELINE config 5 (every rank's observations into one GPU over xGMI). Format:
// wire.h.
//
// The native layout (SPEC §8b: 9,552 B per agent + 32 KB per env) is what the learner reads, but
// most of its bytes are padding a transfer can drop: Entity rows past the visible ones, empty
// inventory slots, Market rows past the listings, one byte per ActionTargets bit, and the Tile
// rows/columns that follow from the window's corner, the Buy.MarketItem mask (a function of the
// listings, the agent's gold and id) and the high nibble of every material: ~0.55 KB per agent
// in the realm in C4 steady state instead of 9,552 B (v2); v3 sends each env's distinct Entity
// rows once, in its entity table, and a 2-B table index per visible row: ~0.3 KB.
//
// Kernels:
//   wire_size / wire_scan / wire_pack   native -> wire (nmmo_wire_pack; counts from the native
//                                       obs launch, no scan of the rows)
//   wire_count (+ wire_scan)            the header of a wire buffer written straight from the
//                                       env state (NMMO_OBS_WIRE; obs_kernel writes the records)
//   wire_unpack                         wire -> native (every byte of the native buffer)
//   wire_check                          header and record-head consistency of a received buffer
//   wire_expand                         wire records -> flat float32 rows (the experience store
//                                       decoding only the rows it keeps, clean_pufferl.py:333-346)
// All HBM-bound byte work.
#include "agent_obs.h"

namespace nmmo {

// per env (128 threads = an agent each): its count words, listings and entity-table rows (the
// distinct ids of its records' Entity rows) into the header, its payload bytes into env_off[e]
__global__ void __launch_bounds__(128) wire_size_kernel(const uint16_t* counts, const int* mcount,
                                                       const uint8_t* native, uint8_t* wire, int n, int P) {
  WireView v = wire_view(wire, n, P);
  __shared__ uint32_t ids[kIdWords];
  __shared__ int pre[kIdWords];
  __shared__ int wsum[16];
  __shared__ int part[2];
  const int e = blockIdx.x, a = threadIdx.x;
  idset_clear(ids);
  __syncthreads();
  int bytes = 0;
  if (a < P) {
    const uint16_t c = counts[(size_t)e * P + a];
    v.cnt[(size_t)e * P + a] = c;
    bytes = wire_record_bytes(c);
    if (c & 0x8000u) {
      const int16_t* ent = reinterpret_cast<const int16_t*>(native + (size_t)e * wire_native_env_bytes(P) +
                                                            (size_t)a * NMMO_NATIVE_ROW_BYTES + NMMO_NATIVE_MASK_BYTES) +
                           kNatI16Entity;
      for (int k = 0; k < (int)(c & 127); k++) idset_add(ids, ent[NMMO_N_ENTITY_COLS * k]);
    }
  }
  for (int o = 32; o > 0; o >>= 1) bytes += __shfl_xor(bytes, o);
  if ((a & 63) == 0) part[a >> 6] = bytes;
  const int ne = idset_prefix(ids, pre, wsum);  // (barriers inside)
  if (a == 0) {
    const int nm = min(max(mcount[e], 0), NMMO_MARKET_ROWS);
    v.mcount[e] = (uint16_t)nm;
    v.ecount[e] = (uint16_t)ne;
    v.env_off[e] = wire_table_bytes(ne) + part[0] + (blockDim.x > 64 ? part[1] : 0) + 32 * nm;
  }
}

// NMMO_OBS_WIRE header from the env state (block per env): per agent in the realm nv =
// entities within the L-inf <= 7 window (itself included; the first 100 in datastore-row order,
// as the obs kernels' compaction), ninv = its occupied inventory prefix; the env's entity table
// (the slots some record shows, ranked by id) into p.wrank[e][slot] (0xFFFF = not in it) and
// ecount[e]; the env's payload bytes into env_off[e] (then wire_scan_kernel); the packed word of
// every datastore row (agent_obs.h ao_pack, with the spawn-immune / dangerous / player bits) into
// p.wpk[e], so the record kernel's workgroups load 2 KB of row words instead of staging the env's
// 24 KB of Entity columns each.
#ifndef NMMO_COUNT_THREADS  // (A/B knob: tools/debug/variants.py)
#define NMMO_COUNT_THREADS 512
#endif
constexpr int kCountThreads = NMMO_COUNT_THREADS;  // a workgroup per env; its agents split over the waves
constexpr int kCountU = (kMaxSlots + kCountThreads - 1) / kCountThreads;  // slots per thread
__global__ void __launch_bounds__(kCountThreads) wire_count_kernel(ObsParams p) {
  __shared__ uint32_t pk[kMaxSlots];         // datastore row - 1 -> ao_pack word (agent_obs.h)
  __shared__ uint32_t pos[kMaxSlots];        // slot -> row << 16 | col (agents' windows)
  __shared__ uint32_t tab[kMaxSlots / 32];   // slots some record shows
  __shared__ uint8_t nin[128];               // occupied inventory prefix per agent
  __shared__ uint32_t ids[kIdWords];
  __shared__ int pre[kIdWords];
  __shared__ int wsum[16];
  __shared__ int bytes;
  constexpr uint32_t kOut = 0xFFFFFFFFu;
  static_assert(kMaxSlots % 64 == 0 && kMaxSlots <= 512 && kIdWords % kCountThreads == 0, "rows per lane; idset");
  WireView v = wire_view(p.wire, p.n_envs, p.P);
  const int e = blockIdx.x, tid = threadIdx.x, lane = lane_id(), S = p.S;
  const int w = __builtin_amdgcn_readfirstlane(wave_id()), nw = blockDim.x >> 6;
  const int16_t* E = p.ent + (size_t)e * NMMO_NF * S;
  int al[kCountU], ds[kCountU], r_[kCountU], c_[kCountU], id_[kCountU], ta_[kCountU], nt_[kCountU];  // slots tid +
#pragma unroll  // kCountThreads u, loaded ahead of the barrier
  for (int u = 0; u < kCountU; u++) {
    const int s = tid + kCountThreads * u;
    al[u] = s < S ? E[F_ALIVE * S + s] : 0;
    ds[u] = s < S ? E[F_DS_ROW * S + s] : 0;
    r_[u] = s < S ? E[F_ROW * S + s] : 0;
    c_[u] = s < S ? E[F_COL * S + s] : 0;
    id_[u] = s < S ? E[F_ID * S + s] : 0;
    ta_[u] = s < S ? E[F_TIME_ALIVE * S + s] : 0;
    nt_[u] = s < S ? E[F_NPC_TYPE * S + s] : 0;
  }
  for (int k = tid; k < kMaxSlots; k += blockDim.x) pk[k] = kOut;
  if (tid < kMaxSlots / 32) tab[tid] = 0u;
  idset_clear(ids);
  if (tid < p.P) {  // the 12 item types of agent tid, loads issued together
    const uint2* it = p.items + ((size_t)e * p.P + tid) * kInv;
    uint32_t ty[kInv];
#pragma unroll
    for (int k = 0; k < kInv; k++) ty[k] = it[k].x & 31u;
    int n = 0;
#pragma unroll
    for (int k = kInv - 1; k >= 0; k--) n = ty[k] ? n + 1 : 0;  // length of the occupied prefix
    nin[tid] = (uint8_t)n;
  }
  if (tid == 0) bytes = 0;
  __syncthreads();
#pragma unroll
  for (int u = 0; u < kCountU; u++) {
    const int s = tid + kCountThreads * u;
    if (s >= kMaxSlots) continue;
    const bool in = s < S && al[u];
    pos[s] = in ? ((uint32_t)(uint16_t)r_[u] << 16) | (uint32_t)(uint16_t)c_[u] : kOut;
    if (in && (unsigned)(ds[u] - 1) < (unsigned)S) {
      const bool player = s < p.P;  // (the flags as agent_obs.h ao_stage)
      pk[ds[u] - 1] = ao_pack(s, r_[u], c_[u], player && ta_[u] < p.spawn_immunity, nt_[u] > 1, player);
    }
  }
  __syncthreads();
  uint32_t pr[kMaxSlots / 64];  // this lane's datastore rows 1 + lane + 64 i
#pragma unroll
  for (int i = 0; i < kMaxSlots / 64; i++) {
    pr[i] = pk[lane + 64 * i];
    if (w == 0) p.wpk[(size_t)e * kMaxSlots + lane + 64 * i] = pr[i];
  }
  int mine = 0;
  for (int a = w; a < p.P; a += nw) {
    const uint32_t pa = pos[a];
    uint32_t word = 0u;
    if (pa != kOut) {  // wave-uniform
      const uint32_t rc = (pa >> 16) | (pa & 0xFFFFu) << 16;  // r | c << 16
      int nvis = 0;
#pragma unroll
      for (int i = 0; i < kMaxSlots / 64; i++) {
        const uint32_t x = pr[i];
        const bool in = ao_in_window(x, rc);  // (an empty row is at (255, 255): outside)
        const uint64_t b = __ballot(in);
        if (in && nvis + __popcll(b & lanes_below()) < kNObs) {
          const int q = ao_slot(x);
          atomicOr(&tab[q >> 5], 1u << (q & 31));
        }
        nvis += __popcll(b);
      }
      word = wire_count_word(min(nvis, kNObs), nin[a]);
    }
    if (lane == 0) {
      v.cnt[(size_t)e * p.P + a] = (uint16_t)word;
      mine += wire_record_bytes(word);
    }
  }
  if (lane == 0) atomicAdd(&bytes, mine);
  __syncthreads();
  bool shown[kCountU];
#pragma unroll
  for (int u = 0; u < kCountU; u++) {
    const int s = tid + kCountThreads * u;
    shown[u] = s < S && ((tab[s >> 5] >> (s & 31)) & 1u);
    if (shown[u]) idset_add(ids, id_[u]);
  }
  const int ne = idset_prefix(ids, pre, wsum);  // (barriers inside)
  uint16_t* rk = p.wrank + (size_t)e * kMaxSlots;
#pragma unroll
  for (int u = 0; u < kCountU; u++) {
    const int s = tid + kCountThreads * u;
    if (s < kMaxSlots) rk[s] = shown[u] ? (uint16_t)idrank(ids, pre, id_[u]) : (uint16_t)0xFFFF;
  }
  if (tid == 0) {
    const int nm = min(max(p.mcount[e], 0), NMMO_MARKET_ROWS);
    v.mcount[e] = (uint16_t)nm;
    v.ecount[e] = (uint16_t)ne;
    v.env_off[e] = wire_table_bytes(ne) + bytes + 32 * nm;
  }
}

// exclusive scan of the per-env payload bytes (one workgroup): env_off[e] becomes the offset of
// env e's payload, *total the buffer size
__global__ void __launch_bounds__(1024) wire_scan_kernel(uint8_t* wire, int n, int P) {
  WireView v = wire_view(wire, n, P);
  __shared__ int64_t wsum[16];
  __shared__ int64_t carry;
  const int tid = threadIdx.x, lane = lane_id(), w = wave_id();
  if (tid == 0) carry = wire_header_bytes(n, P);
  __syncthreads();
  for (int b0 = 0; b0 < n; b0 += 1024) {
    const int e = b0 + tid;
    const int64_t x = e < n ? v.env_off[e] : 0;
    int64_t inc = x;  // inclusive wave scan
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t y = __shfl_up(inc, o);
      if (lane >= o) inc += y;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    int64_t before = carry;
    for (int k = 0; k < w; k++) before += wsum[k];
    if (e < n) v.env_off[e] = before + inc - x;
    __syncthreads();
    if (tid == 1023) carry = before + inc;
    __syncthreads();
  }
  if (tid == 0) *v.total = carry;
  const int64_t used = wire_header_used(n, P);  // header pad is zero
  if (used + tid < wire_header_bytes(n, P)) wire[used + tid] = 0;
}

constexpr int kWireAgentsPerBlock = 16;

__global__ void __launch_bounds__(256) wire_pack_kernel(const uint8_t* native, uint8_t* wire, int n, int P,
                                                        const int16_t* ent, int S, int exch) {
  WireView v = wire_view(wire, n, P);
  __shared__ int off[129];
  __shared__ uint32_t ids[kIdWords];
  __shared__ int pre[kIdWords];
  __shared__ int wsum[16];
  const int e = blockIdx.x, g = blockIdx.y, tid = threadIdx.x, lane = lane_id(), w = wave_id();
  const uint16_t* cnt = v.cnt + (size_t)e * P;
  const int ne = v.ecount[e];
  record_offsets_wave0(cnt, P, off, wire_table_bytes(ne));
  const uint8_t* nenv = native + (size_t)e * wire_native_env_bytes(P);
  auto ent16 = [&](int a) {
    return reinterpret_cast<const int16_t*>(nenv + (size_t)a * NMMO_NATIVE_ROW_BYTES + NMMO_NATIVE_MASK_BYTES) +
           kNatI16Entity;
  };
  // the env's id set again (every block of the env: the table ranks)
  idset_clear(ids);
  __syncthreads();
  for (int a = tid; a < P; a += blockDim.x) {
    const uint32_t c = cnt[a];
    if (!(c & 0x8000u)) continue;
    const int16_t* e16 = ent16(a);
    for (int k = 0; k < (int)(c & 127); k++) idset_add(ids, e16[NMMO_N_ENTITY_COLS * k]);
  }
  idset_prefix(ids, pre, wsum);  // (barriers inside; also publishes off)
  uint8_t* penv = v.base + v.env_off[e];
  if (g == 0) {
    const int nm = v.mcount[e];  // listings: 32 B each, 16-B copies
    const uint4* src = reinterpret_cast<const uint4*>(nenv + (size_t)P * NMMO_NATIVE_ROW_BYTES);
    uint4* dst = reinterpret_cast<uint4*>(penv + off[P]);
    for (int k = tid; k < 2 * nm; k += blockDim.x) dst[k] = src[k];
    // the entity table: every agent's Entity rows to their id's slot (an entity seen twice writes
    // the same bytes twice), wave per agent, int16 per lane; then the table's zero pad
    int16_t* tab = reinterpret_cast<int16_t*>(penv);
    for (int a = w; a < P; a += blockDim.x >> 6) {
      const uint32_t c = cnt[a];
      if (!(c & 0x8000u)) continue;
      const int16_t* e16 = ent16(a);
      for (int j = lane; j < (int)(c & 127) * NMMO_N_ENTITY_COLS; j += 64) {
        const int k = j / NMMO_N_ENTITY_COLS, f = j - k * NMMO_N_ENTITY_COLS;
        tab[idrank(ids, pre, e16[NMMO_N_ENTITY_COLS * k]) * NMMO_N_ENTITY_COLS + f] = e16[j];
      }
    }
    for (int b = kEntRow * ne + tid; b < wire_table_bytes(ne); b += blockDim.x) penv[b] = 0;
  }
  for (int i = w; i < kWireAgentsPerBlock; i += 4) {
    const int a = g * kWireAgentsPerBlock + i;
    if (a >= P) break;
    const uint32_t c = cnt[a];
    if (!(c & 0x8000u)) continue;
    const int nv = c & 127, ninv = (c >> 7) & 15;
    const uint8_t* row = nenv + (size_t)a * NMMO_NATIVE_ROW_BYTES;
    const int16_t* i16 = reinterpret_cast<const int16_t*>(row + NMMO_NATIVE_MASK_BYTES);
    uint8_t* rec = penv + off[a];
    // the ActionTargets as wire.h v4 builds them: head words m5 / m6 from the closed-form
    // sections, the target / inventory entries as a bit stream (ballots over the native bytes)
    const bool style = row[kMkStyle] != 0;
    uint32_t move = 0u;
    for (int k = 0; k < 5; k++) move |= row[kMkMove + k] ? 1u << k : 0u;
    const int ng = __popcll(__ballot(lane < 64 && row[kMkGoldP + lane])) +
                   __popcll(__ballot(lane + 64 < kSecN[6] && row[kMkGoldP + 64 + lane]));
    int pp1 = 0;
    if (exch) {
      const uint64_t z0 = __ballot(!row[kMkSellP + lane]);
      const uint64_t z1 = __ballot(lane + 64 < kSecN[10] && !row[kMkSellP + 64 + lane]);
      pp1 = z0 ? __builtin_ctzll(z0) + 1 : z1 ? 65 + __builtin_ctzll(z1) : 0;
    }
    if (lane == 0) {
      const int gold = ent[((size_t)e * NMMO_NF + F_GOLD) * S + a];  // the state the obs was taken from
      const uint4 head = make_uint4((uint32_t)(uint16_t)i16[0] | (uint32_t)(uint16_t)i16[1] << 16,
                                    (uint32_t)(uint16_t)i16[kNatI16Task] | (uint32_t)(uint16_t)i16[kNatI16Tile] << 16,
                                    (uint32_t)(uint16_t)i16[kNatI16Tile + 1] | wire_m5(nv, ninv, exch, pp1) << 16,
                                    wire_m6(style, move, ng, pp1) | (uint32_t)(uint16_t)gold << 16);
      *reinterpret_cast<uint4*>(rec) = head;
    }
    uint16_t* d16 = reinterpret_cast<uint16_t*>(rec + kWireHead);
    for (int k = lane; k < nv; k += 64) d16[k] = (uint16_t)idrank(ids, pre, i16[kNatI16Entity + NMMO_N_ENTITY_COLS * k]);
    int16_t* s16 = reinterpret_cast<int16_t*>(d16 + nv);
    for (int k = lane; k < ninv * 16; k += 64) s16[k] = i16[kNatI16Inv + k];
    uint8_t* mat = reinterpret_cast<uint8_t*>(s16 + ninv * 16);
    auto tile = [&](int t) { return t < 225 ? (int)i16[kNatI16Tile + 3 * t + 2] & 15 : 0; };
    for (int u = lane; u < kWireTiles; u += 64) mat[u] = (uint8_t)(tile(2 * u) | tile(2 * u + 1) << 4);
    // the stream: bit i of AttackTarget / GiveTarget / GoldTarget (i < nv), then Destroy / GiveItem /
    // SellItem / Use (i < ninv); a lane per bit, a byte per 8 lanes, then the zero pad
    uint8_t* st = mat + kWireTiles;
    const int B = 3 * nv + 4 * ninv, pad = wire_record_bytes(c) - wire_off_stream(nv, ninv);
    for (int i0 = 0; i0 < 8 * pad; i0 += 64) {
      const int i = i0 + lane;
      int k = i, sec;
      if (k < 3 * nv) {
        sec = k / max(nv, 1);
        k -= sec * nv;
        sec = sec == 0 ? kMkAttackT : sec == 1 ? kMkGiveT : kMkGoldT;
      } else {
        k -= 3 * nv;
        const int q = min(k / max(ninv, 1), 3);
        k -= q * ninv;
        sec = q == 0 ? kMkDestroy : q == 1 ? kMkGiveI : q == 2 ? kMkSellI : kMkUse;
      }
      const uint64_t b = __ballot(i < B && row[sec + k] != 0);
      if ((lane & 7) == 0 && i < 8 * pad) st[i >> 3] = (uint8_t)(b >> lane);
    }
  }
}

// One wave's copy of a record into its LDS buffer: every load issued before the first store
// (vmcnt retires in issue order, so loads between stores would wait for them), then the
// release / wave barrier / acquire sequence that hands the bytes to the other lanes.
__device__ __forceinline__ void record_to_lds(const uint8_t* src, int nq, uint4* lrec) {
  const int lane = lane_id();
  const uint4* src4 = reinterpret_cast<const uint4*>(src);
  constexpr int kPer = (kRecMaxU4 + 63) / 64;
  uint4 r[kPer];
#pragma unroll
  for (int k = 0; k < kPer; k++) r[k] = lane + 64 * k < nq ? src4[lane + 64 * k] : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
  for (int k = 0; k < kPer; k++)
    if (lane + 64 * k < nq) lrec[lane + 64 * k] = r[k];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// ... and before the next record overwrites the buffer (every lane's reads of this one done)
__device__ __forceinline__ void record_release() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// wire -> native: every byte of the native buffer is written. Each wave first copies its
// agent's record into LDS, then writes the 9,552-B row with 16-B stores computed from LDS; the
// Buy.MarketItem bytes come from the env's listings (price | owner, staged once per block).
__global__ void __launch_bounds__(256) wire_unpack_kernel(const uint8_t* wire, uint8_t* native, int n, int P) {
  WireView v = wire_view(const_cast<uint8_t*>(wire), n, P);
  __shared__ int off[129];
  __shared__ uint32_t lpo[NMMO_MARKET_ROWS];
  __shared__ uint4 recbuf[4][kRecMaxU4];
  __shared__ uint4 tab4[kMaxSlots * kEntRow / 16];  // the env's entity table
  const int e = blockIdx.x, g = blockIdx.y, lane = lane_id(), w = wave_id();
  const uint16_t* cnt = v.cnt + (size_t)e * P;
  const int ne = min((int)v.ecount[e], kMaxSlots);
  record_offsets_wave0(cnt, P, off, wire_table_bytes(ne));
  __syncthreads();
  uint8_t* nenv = native + (size_t)e * wire_native_env_bytes(P);
  const uint8_t* penv = v.base + v.env_off[e];
  const int nm = v.mcount[e];
  for (int k = threadIdx.x; k < wire_table_bytes(ne) / 16; k += blockDim.x) tab4[k] = reinterpret_cast<const uint4*>(penv)[k];
  const int16_t* tab = reinterpret_cast<const int16_t*>(tab4);
  {
    const int16_t* lst = reinterpret_cast<const int16_t*>(penv + off[P]);
    for (int k = threadIdx.x; k < nm; k += blockDim.x)
      lpo[k] = (uint32_t)(uint16_t)lst[16 * k + 15] | (uint32_t)(uint16_t)lst[16 * k + 2] << 16;
  }
  if (g == 0) {
    const uint4* src = reinterpret_cast<const uint4*>(penv + off[P]);
    uint4* dst = reinterpret_cast<uint4*>(nenv + (size_t)P * NMMO_NATIVE_ROW_BYTES);
    for (int k = threadIdx.x; k < NMMO_NATIVE_MARKET_BYTES / 16; k += blockDim.x)
      dst[k] = k < 2 * nm ? src[k] : make_uint4(0u, 0u, 0u, 0u);
  }
  __syncthreads();
  uint4* lrec = recbuf[w];
  const uint8_t* lb = reinterpret_cast<const uint8_t*>(lrec);
  for (int i = w; i < kWireAgentsPerBlock; i += 4) {
    const int a = g * kWireAgentsPerBlock + i;
    if (a >= P) break;
    const uint32_t c = cnt[a];
    uint4* row4 = reinterpret_cast<uint4*>(nenv + (size_t)a * NMMO_NATIVE_ROW_BYTES);
    if (!(c & 0x8000u)) {
      for (int k = lane; k < NMMO_NATIVE_ROW_BYTES / 16; k += 64) row4[k] = make_uint4(0u, 0u, 0u, 0u);
      continue;
    }
    const int nv = c & 127, ninv = (c >> 7) & 15;
    record_to_lds(penv + off[a], wire_record_bytes(c) / 16, lrec);
    const int16_t* h16 = reinterpret_cast<const int16_t*>(lb);
    const uint16_t* idx = reinterpret_cast<const uint16_t*>(lb + kWireHead);
    const int16_t* s16 = reinterpret_cast<const int16_t*>(lb + wire_off_inv(nv));  // Inventory rows
    const uint8_t* mat = lb + wire_off_mat(nv, ninv);
    const uint8_t* st = lb + wire_off_stream(nv, ninv);  // the mask bit stream
    const int r0 = h16[3], c0 = h16[4], task = h16[2];
    // mask bytes, 16 per lane (1,600 bytes = 100 stores)
    for (int k = lane; k < NMMO_NATIVE_MASK_BYTES / 16; k += 64) {
      uint32_t q[4];
#pragma unroll
      for (int j = 0; j < 4; j++) {
        uint32_t wd = 0u;
#pragma unroll
        for (int b = 0; b < 4; b++) {
          const int x = 16 * k + 4 * j + b;
          wd |= (x < kMaskN && wire_mask_entry_any(x, h16, st, nv, ninv, nm, lpo) ? 1u : 0u) << (8 * b);
        }
        q[j] = wd;
      }
      row4[k] = make_uint4(q[0], q[1], q[2], q[3]);
    }
    auto val = [&](int k) -> uint32_t {
      int x;
      if (k < kNatI16Entity) {
        x = h16[k];
      } else if (k < kNatI16Inv) {
        const int j = k - kNatI16Entity, row = j / NMMO_N_ENTITY_COLS;
        x = row < nv ? tab[min((int)idx[row], kMaxSlots - 1) * NMMO_N_ENTITY_COLS + j - row * NMMO_N_ENTITY_COLS] : 0;
      } else if (k < kNatI16Tile) {
        const int j = k - kNatI16Inv;
        x = j < ninv * 16 ? s16[j] : 0;
      } else if (k < kNatI16Task) {
        const int j = k - kNatI16Tile, t = j / 3, comp = j - 3 * t;
        x = comp == 0 ? r0 + t / 15 : comp == 1 ? c0 + t % 15 : wire_tile(mat, t);
      } else {
        x = k == kNatI16Task ? task : 0;
      }
      return (uint32_t)(uint16_t)x;
    };
    // the int16 part, 8 entries per lane per pass (16-B stores)
    uint4* d4 = reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(row4) + NMMO_NATIVE_MASK_BYTES);
    for (int q = lane; q < NMMO_NATIVE_I16 / 8; q += 64) {
      const int k = 8 * q;
      d4[q] = make_uint4(val(k) | val(k + 1) << 16, val(k + 2) | val(k + 3) << 16, val(k + 4) | val(k + 5) << 16,
                         val(k + 6) | val(k + 7) << 16);
    }
    record_release();
  }
}

__global__ void __launch_bounds__(64 * kCheckEnvsPerBlock) wire_check_kernel(const uint8_t* wire, int n, int P,
                                                                            const int64_t* expect_total, int* status) {
  const int e = blockIdx.x * kCheckEnvsPerBlock + wave_id();
  if (e >= n) return;
  const int bad = wire_check_env(wire, n, P, expect_total, e);
  if (bad) atomicOr(status, bad);
}
// Every received buffer of a step in one launch: grid (max envs, buffers)
__global__ void __launch_bounds__(64 * kCheckEnvsPerBlock) wire_check_many_kernel(WireCheckBatch b, int P,
                                                                                 int* status) {
  const int i = blockIdx.y, e = blockIdx.x * kCheckEnvsPerBlock + wave_id();
  if (e >= b.n[i]) return;
  const int bad = wire_check_env(b.wire[i], b.n[i], P, b.expect[i], e);
  if (bad) atomicOr(status, bad);
}

// Wire records -> flat float32 rows (the pufferlib row of SPEC §8; bit-identical to
// expand_kernel over the unpacked native layout): grid (env, 16-agent group), the env's Market
// rows staged in LDS, one wave per agent row. row_map as in expand_kernel: flat row of agent
// e*P + a, < 0 = not kept (the experience store decodes only the rows it keeps).
__global__ void __launch_bounds__(256) wire_expand_kernel(ObsParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  int16_t* mk = reinterpret_cast<int16_t*>(smem);                         // [1024][16]
  int* off = reinterpret_cast<int*>(smem + NMMO_MARKET_ROWS * 32);        // [P + 1]
  uint4* recbuf = reinterpret_cast<uint4*>(smem + NMMO_MARKET_ROWS * 32 + 144 * 4);  // [4][kRecMaxU4]
  uint4* tab4 = recbuf + 4 * kRecMaxU4;  // the env's entity table
  const int P = p.P, e = blockIdx.x, g = blockIdx.y, tid = threadIdx.x, lane = lane_id(), w = wave_id();
  WireView v = wire_view(p.wire, p.n_envs, P);
  const uint16_t* cnt = v.cnt + (size_t)e * P;
  const int ne = min((int)v.ecount[e], kMaxSlots);
  record_offsets_wave0(cnt, P, off, wire_table_bytes(ne));
  __syncthreads();
  const uint8_t* penv = v.base + v.env_off[e];
  const int nm = v.mcount[e];
  for (int k = tid; k < wire_table_bytes(ne) / 16; k += blockDim.x) tab4[k] = reinterpret_cast<const uint4*>(penv)[k];
  const int16_t* tab = reinterpret_cast<const int16_t*>(tab4);
  {
    const uint4* src = reinterpret_cast<const uint4*>(penv + off[P]);
    uint4* dst = reinterpret_cast<uint4*>(mk);
    for (int k = tid; k < NMMO_MARKET_ROWS * 2; k += blockDim.x) dst[k] = k < 2 * nm ? src[k] : make_uint4(0u, 0u, 0u, 0u);
  }
  __syncthreads();
  uint4* lrec = recbuf + w * kRecMaxU4;
  const uint8_t* lb = reinterpret_cast<const uint8_t*>(lrec);
  for (int i = w; i < kWireAgentsPerBlock; i += 4) {
    const int a = g * kWireAgentsPerBlock + i;
    if (a >= P) break;
    const int frow = p.row_map ? p.row_map[(size_t)e * P + a] : e * P + a;
    if (frow < 0) continue;  // wave-uniform
    float* row = p.obs + (size_t)frow * p.elems;
    const uint32_t c = cnt[a];
    if (!(c & 0x8000u)) {  // not in the realm: all-zero row
      wave_zero(row, 0, p.elems);
      continue;
    }
    const int nv = c & 127, ninv = (c >> 7) & 15;
    record_to_lds(penv + off[a], wire_record_bytes(c) / 16, lrec);
    const int16_t* h16 = reinterpret_cast<const int16_t*>(lb);
    const uint16_t* idx = reinterpret_cast<const uint16_t*>(lb + kWireHead);
    const int16_t* s16 = reinterpret_cast<const int16_t*>(lb + wire_off_inv(nv));  // Inventory rows
    const uint8_t* mat = lb + wire_off_mat(nv, ninv);
    const uint8_t* st = lb + wire_off_stream(nv, ninv);
    const bool exch = wire_exch(h16);
    const int gold = h16[7], aid = h16[0];
    for (int j = lane; j < p.o_agent_id; j += 64) {
      bool m;
      if (j >= kWireBuyLo && j < kWireBuyLo + kWireBuyN) {  // Buy.MarketItem from the staged listings
        const int k = j - kWireBuyLo;
        m = k == NMMO_MARKET_ROWS || (exch && k < nm && mk[16 * k + 15] <= gold && mk[16 * k + 2] != aid);
      } else {
        m = wire_mask_entry(j, h16, st, nv, ninv);
      }
      row[j] = m ? 1.f : 0.f;
    }
    if (lane == 0) row[p.o_agent_id] = (float)h16[0];
    if (lane == 1) row[p.o_tick] = (float)h16[1];
    for (int j = lane; j < kNObs * NMMO_N_ENTITY_COLS; j += 64) {
      const int k = j / NMMO_N_ENTITY_COLS;
      row[p.o_entity + j] =
          k < nv ? (float)tab[min((int)idx[k], kMaxSlots - 1) * NMMO_N_ENTITY_COLS + j - k * NMMO_N_ENTITY_COLS] : 0.f;
    }
    for (int j = lane; j < kInv * 16; j += 64) row[p.o_inventory + j] = j < ninv * 16 ? (float)s16[j] : 0.f;
    for (int j = lane; j < NMMO_MARKET_ROWS * 16; j += 64) row[p.o_market + j] = (float)mk[j];
    const float* temb = p.task + (size_t)h16[2] * p.task_dim;
    for (int j = lane; j < p.task_dim; j += 64) row[p.o_task + j] = temb[j];
    const int r0 = h16[3], c0 = h16[4];
    for (int j = lane; j < 225 * 3; j += 64) {
      const int t = j / 3, comp = j - 3 * t;
      row[p.o_tile + j] = comp == 0 ? (float)(r0 + t / 15) : comp == 1 ? (float)(c0 + t % 15) : (float)wire_tile(mat, t);
    }
    record_release();
  }
}

// Flat rows of record-stored experience rows (nmmo_exp_gather_records): one wave per output row,
// whose record may sit in any stored buffer and env, so nothing is staged per workgroup: the
// wave finds the record (its env's count words -> offsets), copies it into its LDS slot and
// writes the row with every value exactly as wire_expand_kernel computes it (entity-table rows,
// listings and the Task embedding read through L2).
__global__ void __launch_bounds__(256) record_gather_kernel(ObsParams p, NmmoRecordStore rs, const int32_t* idx, int n,
                                                            float* out) {
  __shared__ uint4 recbuf[4][kRecMaxU4];
  const int k = blockIdx.x * 4 + wave_id(), lane = lane_id();
  if (k >= n) return;
  const int s = idx[k];
  const uint8_t* d = rs.arena + rs.row_buf[s];
  const int n_envs = (int)reinterpret_cast<const int64_t*>(d)[0], P = (int)reinterpret_cast<const int64_t*>(d)[1];
  const int ra = rs.row_agent[s], e = ra / P, a = ra - e * P;
  WireView v = wire_view(const_cast<uint8_t*>(d + 16), n_envs, P);
  const uint16_t* cnt = v.cnt + (size_t)e * P;
  const int ne = min((int)v.ecount[e], kMaxSlots), nm = v.mcount[e];
  const uint8_t* penv = v.base + v.env_off[e];
  float* row = out + (size_t)k * p.elems;
  const uint32_t c = cnt[a];
  if (!(c & 0x8000u)) {  // not in the realm: all-zero row
    wave_zero(row, 0, p.elems);
    return;
  }
  // record offset (agents before a) and the listings' offset (all agents), after the table
  int before = 0, all = 0;
  for (int b = 0; b < P; b += 64) {
    const int q = b + lane;
    const int x = q < P ? wire_record_bytes(cnt[q]) : 0;
    before += q < a ? x : 0;
    all += x;
  }
  before = wave_sum(before);
  all = wave_sum(all);
  const int tb = wire_table_bytes(ne);
  const int16_t* tab = reinterpret_cast<const int16_t*>(penv);
  const int16_t* mk = reinterpret_cast<const int16_t*>(penv + tb + all);  // listings, 16 int16 each
  uint4* lrec = recbuf[wave_id()];
  const uint8_t* lb = reinterpret_cast<const uint8_t*>(lrec);
  const int nv = c & 127, ninv = (c >> 7) & 15;
  record_to_lds(penv + tb + before, wire_record_bytes(c) / 16, lrec);
  const int16_t* h16 = reinterpret_cast<const int16_t*>(lb);
  const uint16_t* ix = reinterpret_cast<const uint16_t*>(lb + kWireHead);
  const int16_t* s16 = reinterpret_cast<const int16_t*>(lb + wire_off_inv(nv));  // Inventory rows
  const uint8_t* mat = lb + wire_off_mat(nv, ninv);
  const uint8_t* st = lb + wire_off_stream(nv, ninv);
  const bool exch = wire_exch(h16);
  const int gold = h16[7], aid = h16[0];
  for (int j = lane; j < p.o_agent_id; j += 64) {
    bool m;
    if (j >= kWireBuyLo && j < kWireBuyLo + kWireBuyN) {  // Buy.MarketItem from the listings
      const int q = j - kWireBuyLo;
      m = q == NMMO_MARKET_ROWS || (exch && q < nm && mk[16 * q + 15] <= gold && mk[16 * q + 2] != aid);
    } else {
      m = wire_mask_entry(j, h16, st, nv, ninv);
    }
    row[j] = m ? 1.f : 0.f;
  }
  if (lane == 0) row[p.o_agent_id] = (float)h16[0];
  if (lane == 1) row[p.o_tick] = (float)h16[1];
  for (int j = lane; j < kNObs * NMMO_N_ENTITY_COLS; j += 64) {
    const int q = j / NMMO_N_ENTITY_COLS;
    row[p.o_entity + j] =
        q < nv ? (float)tab[min((int)ix[q], kMaxSlots - 1) * NMMO_N_ENTITY_COLS + j - q * NMMO_N_ENTITY_COLS] : 0.f;
  }
  for (int j = lane; j < kInv * 16; j += 64) row[p.o_inventory + j] = j < ninv * 16 ? (float)s16[j] : 0.f;
  for (int j = lane; j < nm * 16; j += 64) row[p.o_market + j] = (float)mk[j];
  wave_zero(row, p.o_market + nm * 16, p.o_task);
  const float* temb = p.task + (size_t)h16[2] * p.task_dim;
  for (int j = lane; j < p.task_dim; j += 64) row[p.o_task + j] = temb[j];
  const int r0 = h16[3], c0 = h16[4];
  for (int j = lane; j < 225 * 3; j += 64) {
    const int t = j / 3, comp = j - 3 * t;
    row[p.o_tile + j] = comp == 0 ? (float)(r0 + t / 15) : comp == 1 ? (float)(c0 + t % 15) : (float)wire_tile(mat, t);
  }
}

hipError_t launch_record_gather(const ObsParams& p, const NmmoRecordStore& rs, const int32_t* idx, int n, float* out,
                                hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (p.o_task != p.o_market + NMMO_MARKET_ROWS * 16) return hipErrorInvalidValue;
  hipLaunchKernelGGL(record_gather_kernel, dim3((n + 3) / 4), dim3(256), 0, s, p, rs, idx, n, out);
  return hipGetLastError();
}

hipError_t launch_wire_pack(const uint16_t* counts, const int* mcount, const uint8_t* native, uint8_t* wire, int n,
                            int P, const int16_t* ent, int S, int exch, hipStream_t s) {
  if (P > 128 || n <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(wire_size_kernel, dim3(n), dim3(128), 0, s, counts, mcount, native, wire, n, P);
  hipLaunchKernelGGL(wire_scan_kernel, dim3(1), dim3(1024), 0, s, wire, n, P);
  hipLaunchKernelGGL(wire_pack_kernel, dim3(n, (P + kWireAgentsPerBlock - 1) / kWireAgentsPerBlock), dim3(256), 0, s,
                     native, wire, n, P, ent, S, exch);
  return hipGetLastError();
}

hipError_t launch_wire_header(const ObsParams& p, hipStream_t s) {
  if (p.P > 128 || p.n_envs <= 0 || p.S > kMaxSlots || !p.wire) return hipErrorInvalidValue;
  if (!p.counted) hipLaunchKernelGGL(wire_count_kernel, dim3(p.n_envs), dim3(kCountThreads), 0, s, p);
  hipLaunchKernelGGL(wire_scan_kernel, dim3(1), dim3(1024), 0, s, p.wire, p.n_envs, p.P);
  return hipGetLastError();
}

hipError_t launch_wire_unpack(const uint8_t* wire, uint8_t* native, int n, int P, hipStream_t s) {
  if (P > 128 || n <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(wire_unpack_kernel, dim3(n, (P + kWireAgentsPerBlock - 1) / kWireAgentsPerBlock), dim3(256), 0,
                     s, wire, native, n, P);
  return hipGetLastError();
}

hipError_t launch_wire_check_many(const WireCheckBatch& b, int P, int* status, hipStream_t s) {
  int mx = 0;
  for (int i = 0; i < b.count; i++) mx = max(mx, b.n[i]);
  if (b.count <= 0 || mx <= 0) return hipSuccess;
  hipLaunchKernelGGL(wire_check_many_kernel, dim3((mx + kCheckEnvsPerBlock - 1) / kCheckEnvsPerBlock, b.count),
                     dim3(64 * kCheckEnvsPerBlock), 0, s, b, P, status);
  return hipGetLastError();
}

hipError_t launch_wire_check(const uint8_t* wire, int n, int P, const int64_t* expect_total, int* status,
                             hipStream_t s) {
  if (P > 128 || n <= 0 || !status) return hipErrorInvalidValue;
  hipLaunchKernelGGL(wire_check_kernel, dim3((n + kCheckEnvsPerBlock - 1) / kCheckEnvsPerBlock),
                     dim3(64 * kCheckEnvsPerBlock), 0, s, wire, n, P, expect_total, status);
  return hipGetLastError();
}

constexpr size_t kWireExpandLds = (size_t)NMMO_MARKET_ROWS * 32 + 144 * 4 + (size_t)4 * kRecMaxU4 * 16 +
                                  (size_t)kMaxSlots * kEntRow;  // 59.6 KB

hipError_t launch_wire_expand(const ObsParams& p, hipStream_t s) {
  if (p.P > 128 || p.n_envs <= 0 || !p.wire || !p.obs) return hipErrorInvalidValue;
  hipLaunchKernelGGL(wire_expand_kernel, dim3(p.n_envs, (p.P + kWireAgentsPerBlock - 1) / kWireAgentsPerBlock),
                     dim3(256), kWireExpandLds, s, p);
  return hipGetLastError();
}

}  // namespace nmmo
