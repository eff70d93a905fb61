// wire.h — the wire format of native observations (SPEC.md §8c), shared by the codec kernels
// (wire.hip), the wire-writing observation gather (obs.hip, NMMO_OBS_WIRE) and the experience
// store that decodes wire records straight into flat rows (wire.hip).
//
//   header  int64 total bytes | int64 env payload offset [n_envs] | u16 agent count word
//           [n_envs][P] (bit 15 in the realm, bits 0-6 visible entities nv, 7-10 items ninv) |
//           u16 market listings [n_envs]; 16-B aligned
//   payload per env: one record per agent in the realm (slot order), then its listings
//   record  16-B head (int16 AgentId, CurrentTick, task index, tile row 0, tile col 0, nv, ninv,
//           0) | 1,586 ActionTargets bits in 208 B | nv Entity rows (31 x int16) | ninv Inventory
//           rows (16 x int16) | 225 window materials (u8) | zero pad to 16 B
//   listing 16 x int16 (the native Market row)
#pragma once

#include "common.h"

namespace nmmo {

constexpr int kWireHead = 16, kWireMask = 208, kWireTiles = 225;
constexpr int kWireBody = kWireHead + kWireMask;  // 224: Entity rows start 16-B aligned
constexpr int kNatI16Entity = 2, kNatI16Inv = kNatI16Entity + kNObs * NMMO_N_ENTITY_COLS,
              kNatI16Tile = kNatI16Inv + kInv * 16, kNatI16Task = kNatI16Tile + 225 * 3;
constexpr int kRecMaxU4 = (kWireBody + 62 * kNObs + 32 * kInv + kWireTiles + 15) / 16;  // 440

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
