// Diagnostic: how many workgroups of a given shape and dynamic LDS size run at once per CU.
// Launches 256 x k workgroups that each spin ~20 us; the launch takes ~one spin per round, so
// the time jumps when k exceeds the resident workgroups per CU.
//   hipcc --offload-arch=gfx950 -O3 tools/occupancy_probe.hip -o /tmp/occ && /tmp/occ
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void spin(float* out, int iters) {
  extern __shared__ float lds[];
  float x = threadIdx.x;
  for (int i = 0; i < iters; i++) x = x * 1.0000001f + 0.5f;
  lds[threadIdx.x] = x;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = lds[(threadIdx.x + 1) % blockDim.x];
}

int main() {
  float* out;
  if (hipMalloc(&out, 4 * 4096 * sizeof(float)) != hipSuccess) return 1;
  for (int lds : {0}) hipFuncSetAttribute((const void*)spin, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipEvent_t t0, t1;
  hipEventCreate(&t0);
  hipEventCreate(&t1);
  const int threads = 384, iters = 20000;
  for (int lds : {20480, 32768, 39936, 40448, 40768, 40960, 41984, 53248}) {
    printf("LDS %6d B:", lds);
    for (int k : {2, 3, 4, 5}) {
      spin<<<256 * k, threads, lds>>>(out, iters);
      hipEventRecord(t0);
      spin<<<256 * k, threads, lds>>>(out, iters);
      hipEventRecord(t1);
      hipEventSynchronize(t1);
      float ms;
      hipEventElapsedTime(&ms, t0, t1);
      printf("  %d/CU %.1f us", k, ms * 1e3);
    }
    int nb = 0;
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)spin, threads, lds);
    printf("  | runtime says %d per CU\n", nb);
  }
  hipFree(out);
  return 0;
}
