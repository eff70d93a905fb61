// wire.h — the wire format of native observations (SPEC.md §8c), shared by the codec kernels
// (wire.hip), the wire-writing observation gather (obs.hip, NMMO_OBS_WIRE) and the experience
// store that decodes wire records straight into flat rows (wire.hip).
//
//   header  int64 total bytes | int64 env payload offset [n_envs] | u16 agent count word
//           [n_envs][P] (bit 15 in the realm, bits 0-6 visible entities nv, 7-10 items ninv) |
//           u16 market listings [n_envs]; 16-B aligned
//   payload per env: one record per agent in the realm (slot order), then its listings
//   record  16-B head (int16 AgentId, CurrentTick, task index, tile row 0, tile col 0, nv,
//           ninv | exchange << 8, gold) | the ActionTargets as bits EXCEPT Buy.MarketItem (561
//           bits in 80 B) | nv Entity rows (31 x int16) | ninv Inventory rows (16 x int16) | the
//           225 window materials, 4 bits each (113 B) | zero pad to 16 B
//   listing 16 x int16 (the native Market row)
// Buy.MarketItem (1,025 of the 1,586 mask entries) is a function of the env's listings, the
// agent's gold and id: entry k < listings = exchange && price_k <= gold && owner_k != AgentId,
// entry 1,024 (noop) = 1, the rest 0 -- the decoders rebuild it.
#pragma once

#include "common.h"

namespace nmmo {

constexpr int kWireHead = 16;
constexpr int kWireBuyLo = 104, kWireBuyN = NMMO_MARKET_ROWS + 1;  // the Buy section's flat mask entries
constexpr int kMaskN = 1586;                                       // ActionTargets entries (flat offset of AgentId)
constexpr int kWireMaskBits = kMaskN - kWireBuyN;                  // 561 sent
constexpr int kWireMask = 80;                                      // their bytes, zero-padded
constexpr int kWireTiles = 113;                                    // 225 materials, two per byte
constexpr int kWireBody = kWireHead + kWireMask;  // 96: Entity rows start 16-B aligned
static_assert(kWireMaskBits <= 8 * kWireMask && kWireBody % 16 == 0, "wire record head");
// flat mask entry of wire bit b (b < kWireMaskBits), and the wire bit of a non-Buy entry
__host__ __device__ inline int wire_bit_entry(int b) { return b < kWireBuyLo ? b : b + kWireBuyN; }
__host__ __device__ inline int entry_wire_bit(int j) { return j < kWireBuyLo ? j : j - kWireBuyN; }
constexpr int kNatI16Entity = 2, kNatI16Inv = kNatI16Entity + kNObs * NMMO_N_ENTITY_COLS,
              kNatI16Tile = kNatI16Inv + kInv * 16, kNatI16Task = kNatI16Tile + 225 * 3;
constexpr int kRecMaxU4 = (kWireBody + 62 * kNObs + 32 * kInv + kWireTiles + 15) / 16;  // 425

__host__ __device__ inline int64_t wire_header_used(int n, int P) {
  return 8 + 8 * (int64_t)n + 2 * (int64_t)n * P + 2 * (int64_t)n;
}
__host__ __device__ inline int64_t wire_header_bytes(int n, int P) { return (wire_header_used(n, P) + 15) & ~(int64_t)15; }
__host__ __device__ inline uint32_t wire_count_word(int nv, int ninv) { return 0x8000u | (uint32_t)nv | (uint32_t)ninv << 7; }
__host__ __device__ inline int wire_record_bytes(uint32_t cnt) {
  if (!(cnt & 0x8000u)) return 0;
  const int nv = cnt & 127, ninv = (cnt >> 7) & 15;
  return (kWireBody + 62 * nv + 32 * ninv + kWireTiles + 15) & ~15;
}
__host__ __device__ inline size_t wire_native_env_bytes(int P) {
  return (size_t)P * NMMO_NATIVE_ROW_BYTES + NMMO_NATIVE_MARKET_BYTES;
}

// Decoding helpers. lpo[k] = price | owner AgentId << 16 of listing k (Market row k's columns 15
// and 2); head = the record's 8 int16.
__device__ inline bool wire_buy_entry(int k, int nm, const uint32_t* lpo, const int16_t* head) {
  if (k == NMMO_MARKET_ROWS) return true;  // noop
  if (k >= nm || !((uint16_t)head[6] >> 8)) return false;
  const uint32_t v = lpo[k];
  return (int)(v & 0xFFFFu) <= head[7] && (int)(v >> 16) != head[0];
}
// flat ActionTargets entry j (< kMaskN) of a record whose mask bits are `bits`
__device__ inline bool wire_mask_entry(int j, const uint32_t* bits, int nm, const uint32_t* lpo, const int16_t* head) {
  if (j >= kWireBuyLo && j < kWireBuyLo + kWireBuyN) return wire_buy_entry(j - kWireBuyLo, nm, lpo, head);
  const int b = entry_wire_bit(j);
  return (bits[b >> 5] >> (b & 31)) & 1u;
}
// window material t (< 225) of a record's 4-bit tile bytes
__device__ inline int wire_tile(const uint8_t* mat, int t) { return (mat[t >> 1] >> (4 * (t & 1))) & 15; }

struct WireView {  // the header fields of a wire buffer of n envs x P agents
  int64_t* total;
  int64_t* env_off;  // [n] payload offsets (relative to the buffer start)
  uint16_t* cnt;     // [n][P]
  uint16_t* mcount;  // [n]
  uint8_t* base;
};
__device__ inline WireView wire_view(uint8_t* w, int n, int P) {
  WireView v;
  v.base = w;
  v.total = reinterpret_cast<int64_t*>(w);
  v.env_off = v.total + 1;
  v.cnt = reinterpret_cast<uint16_t*>(v.env_off + n);
  v.mcount = v.cnt + (size_t)n * P;
  return v;
}

// Offsets of the records of one env's agents (relative to the env payload) into off[0..P), the
// listings' offset into off[P]. Wave 0 of the block computes them; the caller's next barrier
// publishes them.
__device__ inline void record_offsets_wave0(const uint16_t* cnt, int P, int* off) {
  if (threadIdx.x >= 64) return;
  const int lane = threadIdx.x;
  int carry = 0;
  for (int b = 0; b < P; b += 64) {
    const int a = b + lane;
    const int x = a < P ? wire_record_bytes(cnt[a]) : 0;
    const int inc = wave_incl_scan(x);
    if (a < P) off[a] = carry + inc - x;
    carry += __builtin_amdgcn_readlane(inc, 63);
  }
  if (lane == 0) off[P] = carry;
}

}  // namespace nmmo
