// vmm_repro.hip — standalone HIP reproducer for the chunk-mapped buffer read-back corruption seen
// in round 4 (tools/debug/dbg_vmm.py through nmmo_dev_alloc / nmmo_dev_free): no
// code of the build, only the HIP virtual-memory calls in the order nmmo_dev_alloc / _free use them.
//
// Per cycle: 4 buffers of different sizes, each a virtual range (hipMemAddressReserve) mapped from
// 64-MB physical chunks (hipMemCreate + hipMemMap per chunk, hipMemSetAccess over the range), filled
// by a kernel with the cycle's value, checked by a kernel (mismatching words counted on the device),
// then freed: device sync, unmap, release the chunks, and (unless `keep`) hipMemAddressFree.
// Variants (argv):
//   unmap=whole|chunk   one hipMemUnmap over the whole range, or one per mapped chunk
//   sync=0|1            hipDeviceSynchronize between the unmaps and the releases
//   free=1|0            hipMemAddressFree the range (0: keep it reserved, as nmmo_dev_free does)
//   cycles=N
//   attrs=1             hipPointerGetAttributes on each new range (what torch does when it wraps a
//                       foreign device pointer: torch.as_tensor over __cuda_array_interface__)
//   tmp=1               each check also hipMallocs a quarter-size temporary, written by a kernel and
//                       kept until the end (torch's caching allocator holding the `b == v` results)
// Prints one line per variant run: cycles, buffers with wrong contents, ranges handed out again.
//   hipcc --offload-arch=gfx950 -O2 tools/vmm_repro.hip -o tools/vmm_repro && tools/vmm_repro unmap=whole
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <set>
#include <vector>

#define CHECK(x)                                                                              \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) {                                                                   \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));      \
      exit(2);                                                                                \
    }                                                                                         \
  } while (0)

__global__ void fill_kernel(uint32_t* p, size_t n, uint32_t v) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = v ^ (uint32_t)i;
}
__global__ void check_kernel(const uint32_t* p, size_t n, uint32_t v, unsigned long long* bad) {
  unsigned long long b = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    b += p[i] != (v ^ (uint32_t)i);
  if (b) atomicAdd(bad, b);
}

struct Buf {
  void* va = nullptr;
  size_t total = 0, chunk = 0;
  std::vector<hipMemGenericAllocationHandle_t> chunks;
};

static Buf alloc_buf(int dev, size_t bytes) {
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = dev;
  size_t gran = 0;
  CHECK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum));
  const size_t want = (size_t)64 << 20;
  Buf b;
  b.chunk = gran > want ? gran : (want / gran) * gran;
  b.total = (bytes + b.chunk - 1) / b.chunk * b.chunk;
  CHECK(hipMemAddressReserve(&b.va, b.total, b.chunk, nullptr, 0));
  for (size_t off = 0; off < b.total; off += b.chunk) {
    hipMemGenericAllocationHandle_t h;
    CHECK(hipMemCreate(&h, b.chunk, &prop, 0));
    b.chunks.push_back(h);
    CHECK(hipMemMap((char*)b.va + off, b.chunk, 0, h, 0));
  }
  hipMemAccessDesc acc = {};
  acc.location = prop.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  CHECK(hipMemSetAccess(b.va, b.total, &acc, 1));
  return b;
}

static void free_buf(Buf& b, bool whole, bool sync, bool free_va) {
  CHECK(hipDeviceSynchronize());
  if (whole) {
    CHECK(hipMemUnmap(b.va, b.total));
  } else {
    for (size_t i = 0; i < b.chunks.size(); i++) CHECK(hipMemUnmap((char*)b.va + i * b.chunk, b.chunk));
  }
  if (sync) CHECK(hipDeviceSynchronize());
  for (auto h : b.chunks) CHECK(hipMemRelease(h));
  if (free_va) CHECK(hipMemAddressFree(b.va, b.total));
  b.chunks.clear();
}

int main(int argc, char** argv) {
  bool whole = true, sync = false, free_va = true, attrs = false, tmp = false;
  int cycles = 48;
  for (int i = 1; i < argc; i++) {
    if (!strcmp(argv[i], "unmap=chunk")) whole = false;
    else if (!strcmp(argv[i], "unmap=whole")) whole = true;
    else if (!strcmp(argv[i], "sync=1")) sync = true;
    else if (!strcmp(argv[i], "free=0")) free_va = false;
    else if (!strcmp(argv[i], "attrs=1")) attrs = true;
    else if (!strcmp(argv[i], "tmp=1")) tmp = true;
    else if (!strncmp(argv[i], "cycles=", 7)) cycles = atoi(argv[i] + 7);
  }
  int dev = 0, vmm = 0;
  CHECK(hipSetDevice(dev));
  CHECK(hipDeviceGetAttribute(&vmm, hipDeviceAttributeVirtualMemoryManagementSupported, dev));
  if (!vmm) {
    printf("no virtual memory management on device %d\n", dev);
    return 0;
  }
  unsigned long long* d_bad;
  CHECK(hipMalloc(&d_bad, 8));
  int bad_bufs = 0, reused = 0;
  unsigned long long bad_words = 0;
  std::set<void*> seen;
  std::vector<void*> temps;
  for (int it = 0; it < cycles; it++) {
    Buf bufs[4];
    for (int k = 0; k < 4; k++) {  // the sizes of dbg_vmm.py: (8 + 7 k + it % 12) << 18 floats
      const size_t bytes = (size_t)(8 + 7 * k + it % 12) << 20;
      bufs[k] = alloc_buf(dev, bytes);
      if (!seen.insert(bufs[k].va).second) reused++;
      if (attrs) {
        hipPointerAttribute_t at;
        CHECK(hipPointerGetAttributes(&at, bufs[k].va));
      }
      hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, 0, (uint32_t*)bufs[k].va, bytes / 4,
                         (uint32_t)(it * 10 + k) * 2654435761u);
    }
    CHECK(hipDeviceSynchronize());
    for (int k = 0; k < 4; k++) {
      const size_t bytes = (size_t)(8 + 7 * k + it % 12) << 20;
      CHECK(hipMemset(d_bad, 0, 8));
      if (tmp) {
        void* t = nullptr;
        const size_t tb = ((bytes / 4) + ((size_t)2 << 20) - 1) & ~(((size_t)2 << 20) - 1);
        CHECK(hipMalloc(&t, tb));
        hipLaunchKernelGGL(fill_kernel, dim3(256), dim3(256), 0, 0, (uint32_t*)t, tb / 4, 0x5A5A5A5Au);
        temps.push_back(t);
      }
      hipLaunchKernelGGL(check_kernel, dim3(1024), dim3(256), 0, 0, (const uint32_t*)bufs[k].va, bytes / 4,
                         (uint32_t)(it * 10 + k) * 2654435761u, d_bad);
      unsigned long long b = 0;
      CHECK(hipMemcpy(&b, d_bad, 8, hipMemcpyDeviceToHost));
      if (b) {
        bad_bufs++;
        bad_words += b;
        printf("cycle %d buffer %d va %p: %llu wrong words\n", it, k, bufs[k].va, b);
      }
    }
    for (int k = 0; k < 4; k++) free_buf(bufs[k], whole, sync, free_va);
  }
  printf("vmm_repro unmap=%s sync=%d free=%d attrs=%d tmp=%d cycles=%d: buffers with wrong contents %d (%llu words), "
         "ranges handed out again %d of %d\n",
         whole ? "whole" : "chunk", (int)sync, (int)free_va, (int)attrs, (int)tmp, cycles, bad_bufs, bad_words, reused, 4 * cycles);
  for (void* t : temps) CHECK(hipFree(t));
  CHECK(hipFree(d_bad));
  return bad_bufs ? 1 : 0;
}
