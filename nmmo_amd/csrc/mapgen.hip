// mapgen.hip — map-bank generator (SPEC.md §3), one workgroup per map.
//
// Replaces nmmo's first-use map generation behind `nmmo.Env(Config)` (PATH_MAPS /
// MAP_FORCE_GENERATION, reinforcement_learning/environment.py:33,41). Integer-only value-noise
// fBm so the bank is bit-identical on any device and in the CPU oracle. The noise field (u16)
// and the noise-pass materials are staged in LDS (51 KB + 25.6 KB) because the per-map
// quantile thresholds and the Fish rule need the whole map before any tile is final.
#include "kernels.h"

namespace nmmo {

__device__ inline uint64_t lattice(uint64_t seed, uint32_t m, uint32_t k, uint32_t gy, uint32_t gx) {
  uint32_t a = h32(m * 0x9E3779B1u + k * 0x85EBCA77u);
  uint32_t b = h32((uint32_t)(seed >> 32) ^ a ^ (gy * 0xC2B2AE3Du) ^ (gx * 0x27D4EB2Fu));
  return h32((uint32_t)seed ^ b) >> 16;
}
__device__ inline uint64_t smooth(uint64_t t) { return (t * t * (196608u - 2 * t)) >> 32; }

__global__ void __launch_bounds__(256) mapgen_kernel(uint64_t seed, uint8_t* __restrict__ bank) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint16_t* noise = reinterpret_cast<uint16_t*>(smem);             // [kTiles]
  uint8_t* base = smem + kTiles * 2;                                 // [kTiles]
  int* hist = reinterpret_cast<int*>(smem + kTiles * 3);             // [256]
  int* bounds = hist + 256;                                          // [3]
  const uint32_t m = blockIdx.x;
  for (int i = threadIdx.x; i < 256; i += blockDim.x) hist[i] = 0;
  __syncthreads();
  const uint64_t amp[5] = {16, 8, 4, 2, 1};
  for (int t = threadIdx.x; t < kTiles; t += blockDim.x) {
    const int y = t / kSize, x = t % kSize;
    uint64_t acc = 0;
#pragma unroll
    for (uint32_t k = 0; k < 5; k++) {
      const uint32_t S = 32u >> k, gy = y / S, gx = x / S;
      const uint64_t sy = smooth(((uint64_t)(y % S) << 16) / S);
      const uint64_t sx = smooth(((uint64_t)(x % S) << 16) / S);
      const uint64_t v00 = lattice(seed, m, k, gy, gx), v01 = lattice(seed, m, k, gy, gx + 1);
      const uint64_t v10 = lattice(seed, m, k, gy + 1, gx), v11 = lattice(seed, m, k, gy + 1, gx + 1);
      const uint64_t a = (v00 * (65536 - sx) + v01 * sx) >> 16;
      const uint64_t b = (v10 * (65536 - sx) + v11 * sx) >> 16;
      acc += amp[k] * ((a * (65536 - sy) + b * sy) >> 16);
    }
    const uint16_t v = (uint16_t)(acc / 31);
    noise[t] = v;
    if (y >= kLo && y <= kHi && x >= kLo && x <= kHi) atomicAdd(&hist[v >> 8], 1);
  }
  __syncthreads();
  if (threadIdx.x == 0) {  // 256-bucket cumulative scan, three quantiles
    int bw = 255, bg = 255, bf = 255, cum = 0;
    for (int b = 0; b < 256; b++) {
      cum += hist[b];
      if (bw == 255 && cum >= 2458) bw = b;
      if (bg == 255 && cum >= 11469) bg = b;
      if (bf == 255 && cum >= 13926) bf = b;
    }
    bounds[0] = bw; bounds[1] = bg; bounds[2] = bf;
  }
  __syncthreads();
  const int bw = bounds[0], bg = bounds[1], bf = bounds[2];
  for (int t = threadIdx.x; t < kTiles; t += blockDim.x) {
    const int b = noise[t] >> 8;
    base[t] = b <= bw ? M_WATER : b <= bg ? M_GRASS : b <= bf ? M_FOILAGE : M_STONE;
  }
  __syncthreads();
  uint8_t* out = bank + (size_t)m * kTiles;
  for (int t = threadIdx.x; t < kTiles; t += blockDim.x) {
    const int y = t / kSize, x = t % kSize;
    int mat = base[t];
    if (y >= 1 && y < kSize - 1 && x >= 1 && x < kSize - 1) {
      const uint32_t r = h32((uint32_t)seed ^ h32(m * 0x9E3779B1u ^ 0xA5A5A5A5u ^ h32((uint32_t)t))) % 1000u;
      if (mat == M_GRASS) {
        if (r < 20) mat = M_TREE;
        else if (r < 35) mat = M_ORE;
        else if (r < 45) mat = M_CRYSTAL;
        else if (r < 60) mat = M_HERB;
      } else if (mat == M_WATER && r < 150) {
        const bool land = !impassable(base[t - kSize]) || !impassable(base[t + kSize]) ||
                          !impassable(base[t - 1]) || !impassable(base[t + 1]);
        if (land) mat = M_FISH;
      }
    }
    if (y < kLo || y > kHi || x < kLo || x > kHi) mat = M_VOID;
    else if (y == kLo || y == kHi || x == kLo || x == kHi) mat = M_GRASS;
    out[t] = (uint8_t)mat;
  }
}

size_t mapgen_lds_bytes() { return (size_t)kTiles * 3 + 260 * 4; }

hipError_t launch_mapgen(uint64_t seed, int map_n, uint8_t* bank, hipStream_t stream) {
  hipLaunchKernelGGL(mapgen_kernel, dim3(map_n), dim3(256), mapgen_lds_bytes(), stream, seed, bank);
  return hipGetLastError();
}

}  // namespace nmmo
