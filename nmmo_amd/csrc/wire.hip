// wire.hip — compact transport encoding of native observations (SPEC.md §8c) for the learner
// gather of BASELINE config 5 (every rank's observations into one GPU over xGMI).
//
// The native layout (SPEC §8b: 9,552 B per agent + 32 KB per env) is what the learner reads, but
// most of its bytes are padding a transfer can drop: Entity rows past the visible ones, empty
// inventory slots, Market rows past the listings, one byte per ActionTargets bit, and the Tile
// rows/columns that follow from the window's corner. A wire buffer keeps only what varies:
//
//   header  int64 total bytes | int64 env payload offset [n_envs] | u16 agent count word
//           [n_envs][P] (bit 15 in the realm, bits 0-6 visible entities nv, 7-10 items ninv) |
//           u16 market listings [n_envs]; 16-B aligned
//   payload per env: one record per agent in the realm (slot order), then its listings
//   record  16-B head (int16 AgentId, CurrentTick, task index, tile row 0, tile col 0, nv, ninv,
//           0) | 1,586 ActionTargets bits in 208 B | nv Entity rows (31 x int16) | ninv Inventory
//           rows (16 x int16) | 225 window materials (u8) | zero pad to 16 B
//   listing 16 x int16 (the native Market row)
//
// ~1.3 KB per agent in C4 steady state instead of 9,552 B. HBM-bound: pack reads the ~2.5 KB of
// the native row the record needs and writes the record; unpack reads the record and writes the
// whole 9,552-B native row. The counts come from the native obs kernel (no scan of the rows).
#include "kernels.h"

namespace nmmo {

constexpr int kWireHead = 16, kWireMask = 208, kWireTiles = 225;
constexpr int kNatI16Entity = 2, kNatI16Inv = kNatI16Entity + kNObs * NMMO_N_ENTITY_COLS,
              kNatI16Tile = kNatI16Inv + kInv * 16, kNatI16Task = kNatI16Tile + 225 * 3;

__host__ __device__ inline int64_t wire_header_bytes(int n, int P) {
  return ((8 + 8 * (int64_t)n + 2 * (int64_t)n * P + 2 * (int64_t)n) + 15) & ~(int64_t)15;
}
__host__ __device__ inline int wire_record_bytes(uint32_t cnt) {
  if (!(cnt & 0x8000u)) return 0;
  const int nv = cnt & 127, ninv = (cnt >> 7) & 15;
  return (kWireHead + kWireMask + 62 * nv + 32 * ninv + kWireTiles + 15) & ~15;
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

// per env: its count words and listings into the header, its payload bytes into env_off[e]
__global__ void __launch_bounds__(128) wire_size_kernel(const uint16_t* counts, const int* mcount, uint8_t* wire,
                                                       int n, int P) {
  WireView v = wire_view(wire, n, P);
  const int e = blockIdx.x, a = threadIdx.x;
  __shared__ int part[2];
  int bytes = 0;
  if (a < P) {
    const uint16_t c = counts[(size_t)e * P + a];
    v.cnt[(size_t)e * P + a] = c;
    bytes = wire_record_bytes(c);
  }
  for (int o = 32; o > 0; o >>= 1) bytes += __shfl_xor(bytes, o);
  if ((a & 63) == 0) part[a >> 6] = bytes;
  __syncthreads();
  if (a == 0) {
    const int nm = min(max(mcount[e], 0), NMMO_MARKET_ROWS);
    v.mcount[e] = (uint16_t)nm;
    v.env_off[e] = part[0] + (blockDim.x > 64 ? part[1] : 0) + 32 * nm;
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
  const int64_t used = 8 + 8 * (int64_t)n + 2 * (int64_t)n * P + 2 * (int64_t)n;  // header pad is zero
  if (used + tid < wire_header_bytes(n, P)) wire[used + tid] = 0;
}

// offsets of the records of env e's agents (relative to the env payload) into off[P]
__device__ inline void record_offsets(const uint16_t* cnt, int P, int* off) {
  const int tid = threadIdx.x;
  if (tid < 64) {
    int carry = 0;
    for (int b = 0; b < P; b += 64) {
      const int a = b + tid;
      const int x = a < P ? wire_record_bytes(cnt[a]) : 0;
      int inc = x;
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(inc, o);
        if (tid >= o) inc += y;
      }
      if (a < P) off[a] = carry + inc - x;
      carry += __shfl(inc, 63);
    }
    if (tid == 0) off[P] = carry;  // listings start
  }
  __syncthreads();
}

constexpr int kWireAgentsPerBlock = 16;

__global__ void __launch_bounds__(256) wire_pack_kernel(const uint8_t* native, uint8_t* wire, int n, int P) {
  WireView v = wire_view(wire, n, P);
  __shared__ int off[129];
  const int e = blockIdx.x, g = blockIdx.y, lane = lane_id(), w = wave_id();
  const uint16_t* cnt = v.cnt + (size_t)e * P;
  record_offsets(cnt, P, off);
  const uint8_t* nenv = native + (size_t)e * wire_native_env_bytes(P);
  uint8_t* penv = v.base + v.env_off[e];
  if (g == 0) {  // listings: 32 B each, 16-B copies
    const int nm = v.mcount[e];
    const uint4* src = reinterpret_cast<const uint4*>(nenv + (size_t)P * NMMO_NATIVE_ROW_BYTES);
    uint4* dst = reinterpret_cast<uint4*>(penv + off[P]);
    for (int k = threadIdx.x; k < 2 * nm; k += blockDim.x) dst[k] = src[k];
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
    if (lane == 0) {
      const uint4 head = make_uint4((uint32_t)(uint16_t)i16[0] | (uint32_t)(uint16_t)i16[1] << 16,
                                    (uint32_t)(uint16_t)i16[kNatI16Task] | (uint32_t)(uint16_t)i16[kNatI16Tile] << 16,
                                    (uint32_t)(uint16_t)i16[kNatI16Tile + 1] | (uint32_t)nv << 16,
                                    (uint32_t)ninv);
      *reinterpret_cast<uint4*>(rec) = head;
    }
    if (lane < kWireMask / 4) {  // 32 mask bytes -> one word of bits (bytes past 1,586 are 0)
      uint32_t bits = 0u;
      if (lane < NMMO_NATIVE_MASK_BYTES / 32) {
        const uint4 q0 = reinterpret_cast<const uint4*>(row)[2 * lane];
        const uint4 q1 = reinterpret_cast<const uint4*>(row)[2 * lane + 1];
        const uint32_t wd[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
#pragma unroll
        for (int k = 0; k < 32; k++) bits |= (((wd[k >> 2] >> (8 * (k & 3))) & 255u) != 0u ? 1u : 0u) << k;
      }
      reinterpret_cast<uint32_t*>(rec + kWireHead)[lane] = bits;
    }
    int16_t* d16 = reinterpret_cast<int16_t*>(rec + kWireHead + kWireMask);
    for (int k = lane; k < nv * NMMO_N_ENTITY_COLS; k += 64) d16[k] = i16[kNatI16Entity + k];
    d16 += nv * NMMO_N_ENTITY_COLS;
    for (int k = lane; k < ninv * 16; k += 64) d16[k] = i16[kNatI16Inv + k];
    uint8_t* mat = reinterpret_cast<uint8_t*>(d16 + ninv * 16);
    const int pad = wire_record_bytes(c) - (kWireHead + kWireMask + 62 * nv + 32 * ninv);
    for (int t = lane; t < pad; t += 64) mat[t] = t < kWireTiles ? (uint8_t)i16[kNatI16Tile + 3 * t + 2] : 0;
  }
}

// wire -> native: every byte of the native buffer is written. Each wave first copies its
// agent's record into LDS (every load issued before the first store: vmcnt retires in issue
// order, so loads between stores would wait for them), then writes the 9,552-B row with 16-B
// stores computed from LDS.
constexpr int kRecMaxU4 = (kWireHead + kWireMask + 62 * kNObs + 32 * kInv + kWireTiles + 15) / 16;  // 440

__global__ void __launch_bounds__(256) wire_unpack_kernel(const uint8_t* wire, uint8_t* native, int n, int P) {
  WireView v = wire_view(const_cast<uint8_t*>(wire), n, P);
  __shared__ int off[129];
  __shared__ uint4 recbuf[4][kRecMaxU4];
  const int e = blockIdx.x, g = blockIdx.y, lane = lane_id(), w = wave_id();
  const uint16_t* cnt = v.cnt + (size_t)e * P;
  record_offsets(cnt, P, off);
  uint8_t* nenv = native + (size_t)e * wire_native_env_bytes(P);
  const uint8_t* penv = v.base + v.env_off[e];
  if (g == 0) {
    const int nm = v.mcount[e];
    const uint4* src = reinterpret_cast<const uint4*>(penv + off[P]);
    uint4* dst = reinterpret_cast<uint4*>(nenv + (size_t)P * NMMO_NATIVE_ROW_BYTES);
    for (int k = threadIdx.x; k < NMMO_NATIVE_MARKET_BYTES / 16; k += blockDim.x)
      dst[k] = k < 2 * nm ? src[k] : make_uint4(0u, 0u, 0u, 0u);
  }
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
    const int nv = c & 127, ninv = (c >> 7) & 15, nq = wire_record_bytes(c) / 16;
    {
      const uint4* src4 = reinterpret_cast<const uint4*>(penv + off[a]);
      constexpr int kPer = (kRecMaxU4 + 63) / 64;
      uint4 r[kPer];
#pragma unroll
      for (int k = 0; k < kPer; k++) r[k] = lane + 64 * k < nq ? src4[lane + 64 * k] : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
      for (int k = 0; k < kPer; k++)
        if (lane + 64 * k < nq) lrec[lane + 64 * k] = r[k];
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    const int16_t* h16 = reinterpret_cast<const int16_t*>(lb);
    const int16_t* s16 = reinterpret_cast<const int16_t*>(lb + kWireHead + kWireMask);
    const uint8_t* mat = lb + kWireHead + kWireMask + 62 * nv + 32 * ninv;
    const int r0 = h16[3], c0 = h16[4], task = h16[2];
    // mask bytes, 16 per lane (1,600 bytes = 100 stores)
    for (int k = lane; k < NMMO_NATIVE_MASK_BYTES / 16; k += 64) {
      const uint32_t bits = (reinterpret_cast<const uint32_t*>(lb + kWireHead)[k >> 1] >> (16 * (k & 1))) & 0xFFFFu;
      uint32_t q[4];
#pragma unroll
      for (int j = 0; j < 4; j++)
        q[j] = ((bits >> (4 * j)) & 1u) | ((bits >> (4 * j + 1)) & 1u) << 8 | ((bits >> (4 * j + 2)) & 1u) << 16 |
               ((bits >> (4 * j + 3)) & 1u) << 24;
      row4[k] = make_uint4(q[0], q[1], q[2], q[3]);
    }
    auto val = [&](int k) -> uint32_t {
      int x;
      if (k < kNatI16Entity) {
        x = h16[k];
      } else if (k < kNatI16Inv) {
        const int j = k - kNatI16Entity;
        x = j < nv * NMMO_N_ENTITY_COLS ? s16[j] : 0;
      } else if (k < kNatI16Tile) {
        const int j = k - kNatI16Inv;
        x = j < ninv * 16 ? s16[nv * NMMO_N_ENTITY_COLS + j] : 0;
      } else if (k < kNatI16Task) {
        const int j = k - kNatI16Tile, t = j / 3, comp = j - 3 * t;
        x = comp == 0 ? r0 + t / 15 : comp == 1 ? c0 + t % 15 : (int)mat[t];
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
    __builtin_amdgcn_wave_barrier();  // the next agent's record overwrites this one
  }
}

hipError_t launch_wire_pack(const uint16_t* counts, const int* mcount, const uint8_t* native, uint8_t* wire, int n,
                            int P, hipStream_t s) {
  if (P > 128 || n <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(wire_size_kernel, dim3(n), dim3(128), 0, s, counts, mcount, wire, n, P);
  hipLaunchKernelGGL(wire_scan_kernel, dim3(1), dim3(1024), 0, s, wire, n, P);
  hipLaunchKernelGGL(wire_pack_kernel, dim3(n, (P + kWireAgentsPerBlock - 1) / kWireAgentsPerBlock), dim3(256), 0, s,
                     native, wire, n, P);
  return hipGetLastError();
}

hipError_t launch_wire_unpack(const uint8_t* wire, uint8_t* native, int n, int P, hipStream_t s) {
  if (P > 128 || n <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(wire_unpack_kernel, dim3(n, (P + kWireAgentsPerBlock - 1) / kWireAgentsPerBlock), dim3(256), 0,
                     s, wire, native, n, P);
  return hipGetLastError();
}

}  // namespace nmmo
