// write_ceiling_probe.hip — how fast can MI355X write HBM at all?  The raster's newest-only
// launch (frame + potential, 17.2 GB at C3) reaches ~7.15 TB/s; this measures pure-store
// ceilings on 2 x 8 GiB of fresh device memory: hipMemsetD32Async (the runtime's fill), one
// flat stream of 16-B stores (plain / nontemporal, 1 or 2 stores per lane per iteration),
// and the raster's two-plane pattern with one plane from hipMalloc and one from VMM.
// Median of 7 timed launches (GB/s).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>
#include <functional>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <bool NT, int V>
__global__ __launch_bounds__(256) void flat(float* __restrict__ p, long n4, int per_block) {
  const long base = (long)blockIdx.x * per_block;
  for (int k = threadIdx.x * V; k < per_block; k += 256 * V) {
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const long i = base + k + v;
      if (i < n4) {
        f32x4 x = {(float)i, 1.f, 2.f, 3.f};
        if (NT) __builtin_nontemporal_store(x, (f32x4*)p + i);
        else ((f32x4*)p)[i] = x;
      }
    }
  }
}

__global__ __launch_bounds__(256) void two(float* __restrict__ a, float* __restrict__ b, long n4, int per_block) {
  const long base = (long)blockIdx.x * per_block;
  for (int k = threadIdx.x; k < per_block; k += 256) {
    const long i = base + k;
    f32x4 x = {(float)i, 1.f, 2.f, 3.f};
    __builtin_nontemporal_store(x, (f32x4*)a + i);
    __builtin_nontemporal_store(x + 1.f, (f32x4*)b + i);
  }
}

static float timeit(double bytes, const std::function<void()>& f) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::vector<float> ms;
  for (int r = 0; r < 8; ++r) {
    CHECK(hipEventRecord(e0));
    f();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float t;
    CHECK(hipEventElapsedTime(&t, e0, e1));
    if (r) ms.push_back(t);
  }
  std::sort(ms.begin(), ms.end());
  return (float)(bytes / (ms[ms.size() / 2] * 1e-3) / 1e9);
}

int main() {
  const size_t S = 8ull << 30;  // one C3 plane
  float* m;
  CHECK(hipMalloc(&m, 2 * S));
  const long n4 = (long)(2 * S / 16);
  printf("hipMemsetD32Async 16 GiB: %.0f GB/s\n",
         timeit(2.0 * S, [&] { CHECK(hipMemsetD32Async((hipDeviceptr_t)m, 0x3f800000u, 2 * S / 4, 0)); }));
  for (int per : {1024, 4096, 16384}) {
    const unsigned blocks = (unsigned)((n4 + per - 1) / per);
    printf("flat per_block=%5d x16B: plain V1 %.0f  nt V1 %.0f  plain V2 %.0f  nt V2 %.0f GB/s\n", per,
           timeit(2.0 * S, [&] { hipLaunchKernelGGL((flat<false, 1>), dim3(blocks), dim3(256), 0, 0, m, n4, per); }),
           timeit(2.0 * S, [&] { hipLaunchKernelGGL((flat<true, 1>), dim3(blocks), dim3(256), 0, 0, m, n4, per); }),
           timeit(2.0 * S, [&] { hipLaunchKernelGGL((flat<false, 2>), dim3(blocks), dim3(256), 0, 0, m, n4, per); }),
           timeit(2.0 * S, [&] { hipLaunchKernelGGL((flat<true, 2>), dim3(blocks), dim3(256), 0, 0, m, n4, per); }));
  }
  // two planes: both halves of the hipMalloc buffer, and hipMalloc + VMM
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  hipMemGenericAllocationHandle_t h;
  CHECK(hipMemCreate(&h, S, &prop, 0));
  void* v = nullptr;
  CHECK(hipMemAddressReserve(&v, S, 4096, nullptr, 0));
  CHECK(hipMemMap(v, S, 0, h, 0));
  hipMemAccessDesc acc = {};
  acc.location = prop.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  CHECK(hipMemSetAccess(v, S, &acc, 1));
  const long p4 = (long)(S / 16);
  for (int per : {1024, 4096, 16384}) {
    const unsigned blocks = (unsigned)((p4 + per - 1) / per);
    printf("two planes per_block=%5d: malloc+malloc %.0f  malloc+vmm %.0f  vmm alone %.0f GB/s\n", per,
           timeit(2.0 * S, [&] { hipLaunchKernelGGL(two, dim3(blocks), dim3(256), 0, 0, m, m + S / 4, p4, per); }),
           timeit(2.0 * S, [&] { hipLaunchKernelGGL(two, dim3(blocks), dim3(256), 0, 0, m, (float*)v, p4, per); }),
           timeit(1.0 * S, [&] { hipLaunchKernelGGL((flat<true, 1>), dim3(blocks), dim3(256), 0, 0, (float*)v, p4, per); }));
  }
  CHECK(hipMemUnmap(v, S));
  CHECK(hipMemAddressFree(v, S));
  CHECK(hipMemRelease(h));
  CHECK(hipFree(m));
  return 0;
}
