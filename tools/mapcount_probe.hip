// mapcount_probe.hip — does the number of virtual mappings of a physical piece change how fast
// it can be written?  The seamless ring's slot 0 is mapped three times (the piece's home mapping,
// ring slot 0 and the alias slot W), every other slot twice, and on three boxes slot 0's newest-
// only raster ran ~10 % slower than the others through EITHER of its ring mappings, and stayed
// slow when its pieces were replaced (profiles/r02_slot0.txt).  Here: 1 GiB pieces (hipMemCreate)
// mapped 1, 2 or 3 times (separate reservations), each mapping timed for
//   dense : one 16-B nontemporal store stream over the piece,
//   pair  : the same stream in lockstep with a hipMalloc partner (the raster's frame + potential),
//   sparse: one 16-B store per 64 KiB page, 64 passes (translation-bound: shows PTE fragment size).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/mapcount_probe tools/mapcount_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <functional>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ __launch_bounds__(256) void one(f32x4* __restrict__ a, long n16) {
  for (long i = (long)blockIdx.x * 4096 + threadIdx.x; i < n16 && i < ((long)blockIdx.x + 1) * 4096; i += 256) {
    const f32x4 x = {0.f, 1.f, 2.f, 3.f};
    __builtin_nontemporal_store(x, a + i);
  }
}

__global__ __launch_bounds__(256) void two(f32x4* __restrict__ a, f32x4* __restrict__ b, long n16) {
  for (long i = (long)blockIdx.x * 4096 + threadIdx.x; i < n16 && i < ((long)blockIdx.x + 1) * 4096; i += 256) {
    const f32x4 x = {0.f, 1.f, 2.f, 3.f};
    __builtin_nontemporal_store(x, a + i);
    __builtin_nontemporal_store(x, b + i);
  }
}

// thread t of pass p writes page (t * 7919 + p * 104729) mod pages: scattered over the piece
__global__ __launch_bounds__(256) void sparse(f32x4* __restrict__ a, long pages, int passes) {
  const long t = (long)blockIdx.x * 256 + threadIdx.x;
  if (t >= pages) return;
  for (int p = 0; p < passes; ++p) {
    const long pg = (t * 7919 + (long)p * 104729) % pages;
    const f32x4 x = {(float)p, 1.f, 2.f, 3.f};
    a[pg * 4096] = x;  // 64 KiB = 4096 float4
  }
}

static float time_ms(const std::function<void()>& f) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::vector<float> ms;
  for (int r = 0; r < 7; ++r) {
    CHECK(hipEventRecord(e0));
    f();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float t;
    CHECK(hipEventElapsedTime(&t, e0, e1));
    if (r) ms.push_back(t);
  }
  std::sort(ms.begin(), ms.end());
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return ms[ms.size() / 2];
}

int main(int argc, char** argv) {
  const size_t S = 1ull << 30;
  const int per_kind = argc > 1 ? atoi(argv[1]) : 4;
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  hipMemAccessDesc acc = {};
  acc.location = prop.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  float* partner = nullptr;
  CHECK(hipMalloc(&partner, S));
  auto map = [&](hipMemGenericAllocationHandle_t h) {
    void* v = nullptr;
    CHECK(hipMemAddressReserve(&v, S, S, nullptr, 0));  // 1 GiB aligned, as the ring maps pieces
    CHECK(hipMemMap(v, S, 0, h, 0));
    CHECK(hipMemSetAccess(v, S, &acc, 1));
    return (f32x4*)v;
  };
  const long n16 = (long)(S / 16), pages = (long)(S >> 16);
  const unsigned blocks = (unsigned)((n16 + 4095) / 4096);
  printf("maps piece mapping  dense_GBs  pair_GBs  sparse_ms\n");
  for (int maps = 1; maps <= 3; ++maps) {
    for (int p = 0; p < per_kind; ++p) {
      hipMemGenericAllocationHandle_t h;
      CHECK(hipMemCreate(&h, S, &prop, 0));
      std::vector<f32x4*> va;
      for (int m = 0; m < maps; ++m) va.push_back(map(h));
      for (int m = 0; m < maps; ++m) {
        const float d = time_ms([&] { hipLaunchKernelGGL(one, dim3(blocks), dim3(256), 0, 0, va[m], n16); });
        const float pr = time_ms([&] { hipLaunchKernelGGL(two, dim3(blocks), dim3(256), 0, 0, va[m], (f32x4*)partner, n16); });
        const float sp = time_ms([&] {
          hipLaunchKernelGGL(sparse, dim3((unsigned)((pages + 255) / 256)), dim3(256), 0, 0, va[m], pages, 64);
        });
        printf("%4d %5d %7d  %9.0f  %8.0f  %9.4f\n", maps, p, m, S / (d * 1e-3) / 1e9, 2.0 * S / (pr * 1e-3) / 1e9, sp);
        fflush(stdout);
      }
    }
  }
  return 0;  // never unmap (the re-map hazard, profiles/r01_ring.txt §3); exit releases everything
}
