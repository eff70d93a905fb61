// wire.h — the wire format of native observations (SPEC.md §8c), shared by the codec kernels
// (wire.hip), the wire-writing observation gather (wire_obs.hip, NMMO_OBS_WIRE) and the experience
// store that decodes wire records straight into flat rows (wire.hip).
//
//   header  int64 total bytes | int64 env payload offset [n_envs] | u16 agent count word
//           [n_envs][P] (bit 15 in the realm, bits 0-6 visible entities nv, 7-10 items ninv) |
//           u16 market listings [n_envs] | u16 entity-table rows [n_envs]; 16-B aligned
//   payload per env: its entity table (the distinct Entity rows its records show, ascending by
//           the 16-bit pattern of their id, 62 B each, zero pad to 16 B), one record per agent
//           in the realm (slot order), then its listings
//   record  16-B head (int16 AgentId, CurrentTick, task index, tile row 0, tile col 0, m5, m6,
//           gold) | nv u16 entity-table indices (the agent's Entity rows in order) | ninv
//           Inventory rows (16 x int16) | the 225 window materials, 4 bits each (114 B, the last
//           byte zero) | the mask bit stream (3 nv + 4 ninv bits in whole u16 words) | zero pad
//           to 16 B
//   listing 16 x int16 (the native Market row)
// The ActionTargets (1,586 entries) travel as what they are made of (v4):
//   m5 = nv | ninv << 7 | Exchange << 11 | (pp1 & 15) << 12
//   m6 = Style (its 3 entries are all 1 or all 0) | Move (5 bits) << 1 | GoldPrice ones (a
//        prefix: count) << 6 | (pp1 >> 4) << 13
//   pp1 = 1 + the SellPrice entry the wrapper cleared (0 = none); SellPrice = Exchange ? every
//        entry but that one : none
//   the stream: AttackTarget, GiveTarget, GoldTarget entries 0..nv-1, then Destroy, GiveItem,
//        SellItem, Use entries 0..ninv-1 (every later entry is 0 and each section's noop 1)
//   Buy.MarketItem (1,025 entries) is a function of the env's listings, the agent's gold and id:
//        entry k < listings = Exchange && price_k <= gold && owner_k != AgentId, entry 1,024
//        (noop) = 1, the rest 0 -- the decoders rebuild it.
// An entity seen by several agents of an env (C4 steady state: 5.1 Entity rows per agent, 1.4
// distinct entities per agent) travels once.
#pragma once

#include "common.h"

namespace nmmo {

constexpr int kWireHead = 16;
constexpr int kWireBuyLo = 104, kWireBuyN = NMMO_MARKET_ROWS + 1;  // the Buy section's flat mask entries
constexpr int kMaskN = 1586;                                       // ActionTargets entries (flat offset of AgentId)
constexpr int kWireTiles = 114;                                    // 225 materials, two per byte (+ a zero byte)
// flat offsets of the ActionTargets sections (nmmo_layout order)
constexpr int kMkStyle = 0, kMkAttackT = 3, kMkDestroy = 1129, kMkGiveI = 1142, kMkGiveT = 1155, kMkGoldP = 1256,
              kMkGoldT = 1355, kMkMove = 1456, kMkSellI = 1461, kMkSellP = 1474, kMkUse = 1573;
constexpr int kNatI16Entity = 2, kNatI16Inv = kNatI16Entity + kNObs * NMMO_N_ENTITY_COLS,
              kNatI16Tile = kNatI16Inv + kInv * 16, kNatI16Task = kNatI16Tile + 225 * 3;
// the mask bit stream: 3 nv + 4 ninv bits in whole u16 words
__host__ __device__ inline int wire_stream_bytes(int nv, int ninv) { return 2 * ((3 * nv + 4 * ninv + 15) >> 4); }
// record offsets (bytes from the record start)
__host__ __device__ inline int wire_off_inv(int nv) { return kWireHead + 2 * nv; }
__host__ __device__ inline int wire_off_mat(int nv, int ninv) { return kWireHead + 2 * nv + 32 * ninv; }
__host__ __device__ inline int wire_off_stream(int nv, int ninv) { return wire_off_mat(nv, ninv) + kWireTiles; }
constexpr int kRecMaxU4 = (kWireHead + 2 * kNObs + 32 * kInv + kWireTiles + 2 * ((3 * kNObs + 4 * kInv + 15) >> 4) +
                           15) / 16;  // 48
constexpr int kEntRow = 2 * NMMO_N_ENTITY_COLS;                                          // 62 B
// head words 5 and 6 (m5, m6 above)
__host__ __device__ inline uint32_t wire_m5(int nv, int ninv, bool exch, int pp1) {
  return (uint32_t)nv | (uint32_t)ninv << 7 | (exch ? 1u << 11 : 0u) | (uint32_t)(pp1 & 15) << 12;
}
__host__ __device__ inline uint32_t wire_m6(bool style, uint32_t move, int ng, int pp1) {
  return (style ? 1u : 0u) | (move & 31u) << 1 | (uint32_t)ng << 6 | (uint32_t)(pp1 >> 4) << 13;
}
__host__ __device__ inline bool wire_exch(const int16_t* head) { return ((uint16_t)head[5] >> 11) & 1u; }
__host__ __device__ inline int wire_pp1(const int16_t* head) {
  return ((uint16_t)head[5] >> 12) | ((uint16_t)head[6] >> 13) << 4;
}

__host__ __device__ inline int64_t wire_header_used(int n, int P) {
  return 8 + 8 * (int64_t)n + 2 * (int64_t)n * P + 4 * (int64_t)n;
}
__host__ __device__ inline int64_t wire_header_bytes(int n, int P) { return (wire_header_used(n, P) + 15) & ~(int64_t)15; }
__host__ __device__ inline uint32_t wire_count_word(int nv, int ninv) { return 0x8000u | (uint32_t)nv | (uint32_t)ninv << 7; }
__host__ __device__ inline int wire_record_bytes(uint32_t cnt) {
  if (!(cnt & 0x8000u)) return 0;
  const int nv = cnt & 127, ninv = (cnt >> 7) & 15;
  return (wire_off_stream(nv, ninv) + wire_stream_bytes(nv, ninv) + 15) & ~15;
}
// an env's entity table of ne rows
__host__ __device__ inline int wire_table_bytes(int ne) { return (kEntRow * ne + 15) & ~15; }
__host__ __device__ inline size_t wire_native_env_bytes(int P) {
  return (size_t)P * NMMO_NATIVE_ROW_BYTES + NMMO_NATIVE_MARKET_BYTES;
}

// Ranks by entity id: the env's distinct ids as a 65,536-bit set (2,048 words in LDS) and the
// exclusive popcount prefix of its words (wave-summed, 2,048 ints); the table index of an id in
// the set is idrank(). Every thread of the block calls the builders (barriers inside).
constexpr int kIdWords = 65536 / 32;
__device__ inline void idset_clear(uint32_t* ids) {
  for (int k = threadIdx.x; k < kIdWords; k += blockDim.x) ids[k] = 0u;
}
__device__ inline void idset_add(uint32_t* ids, int id) {
  const uint32_t u = (uint16_t)id;
  atomicOr(&ids[u >> 5], 1u << (u & 31));
}
// pre[k] = set ids below word k; returns the set's size (every thread). Needs blockDim.x a
// multiple of 64 dividing kIdWords; wsum >= 16 ints.
__device__ inline int idset_prefix(const uint32_t* ids, int* pre, int* wsum) {
  __syncthreads();
  const int nt = blockDim.x, per = kIdWords / nt, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int loc = 0;
  for (int j = 0; j < per; j++) loc += __popc(ids[tid * per + j]);
  const int inc = wave_incl_scan(loc);
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  int before = 0, total = 0;
  for (int k = 0; k < (nt >> 6); k++) {
    before += k < w ? wsum[k] : 0;
    total += wsum[k];
  }
  int run = before + inc - loc;
  for (int j = 0; j < per; j++) {
    pre[tid * per + j] = run;
    run += __popc(ids[tid * per + j]);
  }
  __syncthreads();
  return total;
}
__device__ inline int idrank(const uint32_t* ids, const int* pre, int id) {
  const uint32_t u = (uint16_t)id;
  return pre[u >> 5] + __popc(ids[u >> 5] & ((1u << (u & 31)) - 1u));
}

// Decoding helpers. lpo[k] = price | owner AgentId << 16 of listing k (Market row k's columns 15
// and 2); head = the record's 8 int16.
__device__ inline bool wire_buy_entry(int k, int nm, const uint32_t* lpo, const int16_t* head) {
  if (k == NMMO_MARKET_ROWS) return true;  // noop
  if (k >= nm || !wire_exch(head)) return false;
  const uint32_t v = lpo[k];
  return (int)(v & 0xFFFFu) <= head[7] && (int)(v >> 16) != head[0];
}
// flat ActionTargets entry j (< kMaskN, not in Buy.MarketItem) of a record: head, its mask bit
// stream (byte pointer), nv, ninv
__device__ inline bool wire_mask_entry(int j, const int16_t* head, const uint8_t* st, int nv, int ninv) {
  const uint32_t m6 = (uint16_t)head[6];
  auto bit = [&](int i) { return ((st[i >> 3] >> (i & 7)) & 1u) != 0; };
  // list sections: entries < n from the stream at s0, the noop (last entry) 1, the rest 0
  auto list = [&](int k, int n, int noop, int s0) { return k == noop ? true : k < n ? bit(s0 + k) : false; };
  if (j < kMkAttackT) return m6 & 1u;                                  // Style
  if (j < kWireBuyLo) return list(j - kMkAttackT, nv, kNObs, 0);       // AttackTarget
  if (j < kMkGiveI) return list(j - kMkDestroy, ninv, kInv, 3 * nv);   // Destroy
  if (j < kMkGiveT) return list(j - kMkGiveI, ninv, kInv, 3 * nv + ninv);  // GiveItem
  if (j < kMkGoldP) return list(j - kMkGiveT, nv, kNObs, nv);          // GiveTarget
  if (j < kMkGoldT) return j - kMkGoldP < (int)((m6 >> 6) & 127u);     // GoldPrice: a prefix of ones
  if (j < kMkMove) return list(j - kMkGoldT, nv, kNObs, 2 * nv);       // GoldTarget
  if (j < kMkSellI) return (m6 >> (1 + j - kMkMove)) & 1u;             // Move
  if (j < kMkSellP) return list(j - kMkSellI, ninv, kInv, 3 * nv + 2 * ninv);  // SellItem
  if (j < kMkUse) return wire_exch(head) && j - kMkSellP + 1 != wire_pp1(head);  // SellPrice
  return list(j - kMkUse, ninv, kInv, 3 * nv + 3 * ninv);             // Use
}
__device__ inline bool wire_mask_entry_any(int j, const int16_t* head, const uint8_t* st, int nv, int ninv, int nm,
                                           const uint32_t* lpo) {
  if (j >= kWireBuyLo && j < kWireBuyLo + kWireBuyN) return wire_buy_entry(j - kWireBuyLo, nm, lpo, head);
  return wire_mask_entry(j, head, st, nv, ninv);
}
// window material t (< 225) of a record's 4-bit tile bytes
__device__ inline int wire_tile(const uint8_t* mat, int t) { return (mat[t >> 1] >> (4 * (t & 1))) & 15; }

struct WireView {  // the header fields of a wire buffer of n envs x P agents
  int64_t* total;
  int64_t* env_off;  // [n] payload offsets (relative to the buffer start)
  uint16_t* cnt;     // [n][P]
  uint16_t* mcount;  // [n]
  uint16_t* ecount;  // [n] entity-table rows
  uint8_t* base;
};
__device__ inline WireView wire_view(uint8_t* w, int n, int P) {
  WireView v;
  v.base = w;
  v.total = reinterpret_cast<int64_t*>(w);
  v.env_off = v.total + 1;
  v.cnt = reinterpret_cast<uint16_t*>(v.env_off + n);
  v.mcount = v.cnt + (size_t)n * P;
  v.ecount = v.mcount + n;
  return v;
}

// Offsets of the records of one env's agents (relative to the env payload, after its entity
// table of `base` bytes) into off[0..P), the listings' offset into off[P]. Wave 0 of the block
// computes them; the caller's next barrier publishes them.
__device__ inline void record_offsets_wave0(const uint16_t* cnt, int P, int* off, int base) {
  if (threadIdx.x >= 64) return;
  const int lane = threadIdx.x;
  int carry = base;
  for (int b = 0; b < P; b += 64) {
    const int a = b + lane;
    const int x = a < P ? wire_record_bytes(cnt[a]) : 0;
    const int inc = wave_incl_scan(x);
    if (a < P) off[a] = carry + inc - x;
    carry += __builtin_amdgcn_readlane(inc, 63);
  }
  if (lane == 0) off[P] = carry;
}

// Consistency of one received wire buffer of n envs x P agents, one wave per env (lane l holds
// agents l and l + 64: the record offsets are two wave scans in registers, no LDS, no barrier):
// the announced total (when expect_total is given), the env payload offsets against the count
// words and listings, the counts' ranges, every record head's AgentId / nv / ninv / closed-form
// mask fields against its count word and its entity-table indices against the table. Returns
// this lane's bits: 1 total, 2 env offsets, 4 count ranges, 8 record heads, 16 entity-table
// indices.
__device__ __forceinline__ int wire_check_env(const uint8_t* wire, int n, int P, const int64_t* expect_total, int e) {
  WireView v = wire_view(const_cast<uint8_t*>(wire), n, P);
  const int lane = threadIdx.x & 63;
  const uint16_t* cnt = v.cnt + (size_t)e * P;
  const uint32_t c0 = lane < P ? cnt[lane] : 0u, c1 = lane + 64 < P ? cnt[lane + 64] : 0u;
  const int ne = v.ecount[e];
  const int64_t total = *v.total;
  const int64_t base = v.env_off[e];
  const int nm = v.mcount[e];
  const int x0 = wire_record_bytes(c0), x1 = wire_record_bytes(c1);
  const int i0 = wave_incl_scan(x0), i1 = wave_incl_scan(x1);
  const int tb = wire_table_bytes(ne), t0 = __builtin_amdgcn_readlane(i0, 63);
  const int all = tb + t0 + __builtin_amdgcn_readlane(i1, 63);  // the listings' offset
  int bad = 0;
  if (lane == 0) {
    if (e == 0 && expect_total && total != *expect_total) bad |= 1;
    if (e == 0 && base != wire_header_bytes(n, P)) bad |= 2;
    const int64_t end = e + 1 < n ? v.env_off[e + 1] : total;
    if (end - base != (int64_t)all + 32 * nm) bad |= 2;
    if (nm > NMMO_MARKET_ROWS || ne > kMaxSlots) bad |= 4;
  }
  auto agent = [&](uint32_t c, int off) {
    int b = 0;
    if (c & 0x8000u) {
      const int nv = c & 127, ninv = (c >> 7) & 15;
      if (nv > kNObs || ninv > kInv || (c & 0x7800u)) {
        b |= 4;
      } else if (base + off + kWireHead <= total) {
        const int16_t* h = reinterpret_cast<const int16_t*>(v.base + base + off);
        if (h[0] <= 0 || ((uint16_t)h[5] & 0x7FFu) != (c & 0x7FFu) || wire_pp1(h) > 99 ||
            (((uint16_t)h[6] >> 6) & 127u) > 99)
          b |= 8;
        if (base + off + wire_record_bytes(c) <= total) {  // entity-table indices, 8 per 16-B load
          const uint4* ix4 = reinterpret_cast<const uint4*>(h + kWireHead / 2);
          uint4 q[(kNObs + 7) / 8];
#pragma unroll
          for (int j = 0; j < (kNObs + 7) / 8; j++) q[j] = 8 * j < nv ? ix4[j] : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
          for (int j = 0; j < (kNObs + 7) / 8; j++) {
            const uint32_t wd[4] = {q[j].x, q[j].y, q[j].z, q[j].w};
#pragma unroll
            for (int i = 0; i < 8; i++)
              if (8 * j + i < nv && ((wd[i >> 1] >> (16 * (i & 1))) & 0xFFFFu) >= (uint32_t)ne) b |= 16;
          }
        }
      } else {
        b |= 2;
      }
    } else if (c) {
      b |= 4;
    }
    return b;
  };
  bad |= agent(c0, tb + i0 - x0);
  bad |= agent(c1, tb + t0 + i1 - x1);
  return bad;
}
constexpr int kCheckEnvsPerBlock = 4;  // one wave per env

}  // namespace nmmo
