// Diagnostic: HBM write rate of the store patterns an obs launch can use, over the C4 obs
// buffer (1024 envs x 128 agents x 23,987 floats = 12.8 GB). Build + run on the GPU box:
//   hipcc --offload-arch=gfx950 -O3 tools/fill_patterns.hip -o /tmp/fill && /tmp/fill
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <vector>

constexpr int kElems = 23987, kEnvs = 1024, kP = 128;

__device__ inline void row_zero(float* row, int lo, int hi, int lane, int nl) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(row + lo);
  int head = (int)(((16 - (a & 15)) & 15) >> 2);
  if (head > hi - lo) head = hi - lo;
  if (lane < head) row[lo + lane] = 0.f;
  const int body = (hi - lo - head) >> 2;
  float4* p4 = reinterpret_cast<float4*>(row + lo + head);
  for (int i = lane; i < body; i += nl) p4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  const int tail0 = lo + head + body * 4;
  if (tail0 + lane < hi) row[tail0 + lane] = 0.f;
}

// (a) grid-stride float4 fill of the whole buffer
__global__ void fill_stride(float4* p, size_t n4) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x)
    p[i] = make_float4(0.f, 0.f, 0.f, 0.f);
}
// (b) the obs grid: (env, 16-agent group), 4 waves, one wave per row, rows w, w+4, w+8, w+12
__global__ void __launch_bounds__(256) fill_row_per_wave(float* obs) {
  const int e = blockIdx.x, g = blockIdx.y, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int i = w; i < 16; i += 4) row_zero(obs + ((size_t)e * kP + g * 16 + i) * kElems, 0, kElems, lane, 64);
}
// (c) same grid, the whole workgroup writes one row at a time
__global__ void __launch_bounds__(256) fill_row_per_block(float* obs) {
  const int e = blockIdx.x, g = blockIdx.y;
  for (int i = 0; i < 16; i++) row_zero(obs + ((size_t)e * kP + g * 16 + i) * kElems, 0, kElems, threadIdx.x, 256);
}
// (d) one wave per row, rows w, w+4, ... but rows of a wave interleaved in 4-KB pieces: the
// 4 waves of a block sweep the block's 16 rows piece by piece together
__global__ void __launch_bounds__(256) fill_row_per_wave_dword(float* obs) {
  const int e = blockIdx.x, g = blockIdx.y, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int i = w; i < 16; i += 4) {
    float* row = obs + ((size_t)e * kP + g * 16 + i) * kElems;
    for (int j = lane; j < kElems; j += 64) row[j] = 0.f;
  }
}
// (e) one wave per row with 8 waves per block (2 rows each)
__global__ void __launch_bounds__(512) fill_row_per_wave8(float* obs) {
  const int e = blockIdx.x, g = blockIdx.y, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int i = w; i < 16; i += 8) row_zero(obs + ((size_t)e * kP + g * 16 + i) * kElems, 0, kElems, lane, 64);
}

// (f) one-shot blocks: 256 threads write 16 KB (4 float4 each, 4 KB per wave-instruction group) and exit
__global__ void __launch_bounds__(256) fill_oneshot(float4* p, size_t n4) {
  const size_t base = (size_t)blockIdx.x * 1024 + threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; i++)
    if (base + 256 * i < n4) p[base + 256 * i] = make_float4(0.f, 0.f, 0.f, 0.f);
}
// (b') the obs rows with the group index fastest in dispatch order (blockIdx.x = group): resident
// workgroups write adjacent 1.5-MB spans
__global__ void __launch_bounds__(256) fill_row_per_wave_gmajor(float* obs) {
  const int g = blockIdx.x, e = blockIdx.y, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int i = w; i < 16; i += 4) row_zero(obs + ((size_t)e * kP + g * 16 + i) * kElems, 0, kElems, lane, 64);
}
// (b'') as (b') with a 1-D grid walked in row order and 8 agents per workgroup (2 per wave)
__global__ void __launch_bounds__(256) fill_row_per_wave_8(float* obs) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const size_t r0 = (size_t)blockIdx.x * 8;
  for (int i = w; i < 8; i += 4) row_zero(obs + (r0 + i) * kElems, 0, kElems, lane, 64);
}
// (g) the obs grid restricted to envs [e0, e0 + ne): a launch per chunk of envs
__global__ void __launch_bounds__(256) fill_row_per_wave_chunk(float* obs, int e0) {
  const int e = e0 + blockIdx.x, g = blockIdx.y, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int i = w; i < 16; i += 4) row_zero(obs + ((size_t)e * kP + g * 16 + i) * kElems, 0, kElems, lane, 64);
}
// (h) torch-like one-shot blocks: T threads, V float4 per thread, block chunk = T*V*16 B, lane-linear
template <int T, int V>
__global__ void __launch_bounds__(T) fill_oneshot_tv(float4* p, size_t n4) {
  const size_t base = (size_t)blockIdx.x * (T * V) + threadIdx.x;
#pragma unroll
  for (int i = 0; i < V; i++)
    if (base + (size_t)T * i < n4) p[base + (size_t)T * i] = make_float4(0.f, 0.f, 0.f, 0.f);
}
// (P4) one workgroup per row (4 waves interleaved 1 KB each, 4 KB steps), workgroups in row order
__global__ void __launch_bounds__(256) fill_wg_per_row(float* obs) {
  row_zero(obs + (size_t)blockIdx.x * kElems, 0, kElems, threadIdx.x, 256);
}
// (P5) one single-wave workgroup per row, in row order
__global__ void __launch_bounds__(64) fill_wave_per_row(float* obs) {
  row_zero(obs + (size_t)blockIdx.x * kElems, 0, kElems, threadIdx.x, 64);
}
// (P6) 4-wave workgroups, wave w writes row 4 * blockIdx.x + w, in row order
__global__ void __launch_bounds__(256) fill_4rows_per_wg(float* obs) {
  row_zero(obs + ((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * kElems, 0, kElems, threadIdx.x & 63, 64);
}
// (P7) as P6 with 16 rows per workgroup (the obs kernel's) but row-ordered grid
__global__ void __launch_bounds__(256) fill_16rows_rowordered(float* obs) {
  const int w = threadIdx.x >> 6;
  for (int i = w; i < 16; i += 4) row_zero(obs + ((size_t)blockIdx.x * 16 + i) * kElems, 0, kElems, threadIdx.x & 63, 64);
}
int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  const size_t n = (size_t)kEnvs * kP * kElems;
  hipEvent_t t0, t1;
  hipEventCreate(&t0);
  hipEventCreate(&t1);
  const dim3 grid(kEnvs, kP / 16);
  auto timeit = [&](const char* name, auto launch) {
    for (int i = 0; i < 3; i++) launch();
    hipEventRecord(t0);
    const int k = 10;
    for (int i = 0; i < k; i++) launch();
    hipEventRecord(t1);
    hipEventSynchronize(t1);
    float ms;
    hipEventElapsedTime(&ms, t0, t1);
    ms /= k;
    printf("%-40s %.3f ms  %.2f TB/s\n", name, ms, n * 4 / (ms * 1e-3) / 1e12);
  };
  auto suite = [&](float* obs, const char* tag) {
    printf("-- %s\n", tag);
    timeit("stride float4 (8192x256)", [&] { fill_stride<<<8192, 256>>>((float4*)obs, n / 4); });
    timeit("row per wave (4 waves)", [&] { fill_row_per_wave<<<grid, 256, 38800>>>(obs); });
    timeit("row per wave, dword stores", [&] { fill_row_per_wave_dword<<<grid, 256, 38800>>>(obs); });
    timeit("row per block", [&] { fill_row_per_block<<<grid, 256>>>(obs); });
  };
  // hipMalloc vs virtual-memory allocations (hipMemCreate chunks mapped into one VA range)
  auto timepat = [&](float* q, const char* tag) {
    printf("%s\n", tag);
    const size_t n4 = n / 4;
    timeit("  rows, one launch (obs shape)", [&] { fill_row_per_wave<<<grid, 256, 38800>>>(q); });
    timeit("  one-shot 256 thr x 1 f4 (4 KB)", [&] { fill_oneshot_tv<256, 1><<<(unsigned)((n4 + 255) / 256), 256>>>((float4*)q, n4); });
  };
  float* bufs[4];
  for (int i = 0; i < 2; i++) {
    if (hipMalloc(&bufs[i], n * 4) != hipSuccess) return 1;
    timepat(bufs[i], "hipMalloc");
  }
  for (int i = 0; i < 2; i++) hipFree(bufs[i]);
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  size_t gran = 0;
  hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended);
  printf("recommended granularity %zu\n", gran);
  for (size_t chunk : {(size_t)2 << 20, (size_t)16 << 20, (size_t)64 << 20, (size_t)256 << 20}) {
    for (int rep = 0; rep < 2; rep++) {
      printf("mapping %zu MB chunks\n", chunk >> 20);
      const size_t total = ((n * 4 + chunk - 1) / chunk) * chunk;
      void* va = nullptr;
      if (hipMemAddressReserve(&va, total, chunk, nullptr, 0) != hipSuccess) { printf("reserve failed\n"); break; }
      std::vector<hipMemGenericAllocationHandle_t> hs;
      bool ok = true;
      for (size_t off = 0; off < total && ok; off += chunk) {
        hipMemGenericAllocationHandle_t h;
        ok = hipMemCreate(&h, chunk, &prop, 0) == hipSuccess &&
             hipMemMap((char*)va + off, chunk, 0, h, 0) == hipSuccess;
        hs.push_back(h);
      }
      hipMemAccessDesc acc = {};
      acc.location = prop.location;
      acc.flags = hipMemAccessFlagsProtReadWrite;
      ok = ok && hipMemSetAccess(va, total, &acc, 1) == hipSuccess;
      char tag[96];
      snprintf(tag, sizeof tag, "VMM chunks of %zu MB (%s)", chunk >> 20, ok ? "ok" : "FAILED");
      if (ok) timepat((float*)va, tag); else printf("%s\n", tag);
      hipMemUnmap(va, total);
      for (auto h : hs) hipMemRelease(h);
      hipMemAddressFree(va, total);
    }
  }
  return 0;
}
