// pair_alias_probe.hip — is the fast/slow pairing of two lockstep write streams a property of
// the PHYSICAL memory or of the VIRTUAL addresses (TLB sets)?  Physical 4 GiB handles H_0..H_15
// (hipMemCreate); H_0 mapped at A; every H_k mapped twice, at B_k and at C_k (two separate
// reservations).  pair(A, B_k) vs pair(A, C_k): same physical pages, different virtual
// addresses.  Also pair(A', B_k) with A' = a second mapping of H_0.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>
#include <functional>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ __launch_bounds__(256) void two(float* __restrict__ a, float* __restrict__ b, int per_block) {
  const long base = (long)blockIdx.x * per_block;
  for (int k = threadIdx.x; k < per_block; k += 256) {
    f32x4 x = {(float)k, 1.f, 2.f, 3.f};
    __builtin_nontemporal_store(x, (f32x4*)a + base + k);
    __builtin_nontemporal_store(x + 1.f, (f32x4*)b + base + k);
  }
}

static float timeit(double bytes, const std::function<void()>& f) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::vector<float> ms;
  for (int r = 0; r < 6; ++r) {
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
  const size_t S = 4ull << 30;
  const int K = 16;
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  hipMemAccessDesc acc = {};
  acc.location = prop.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  std::vector<hipMemGenericAllocationHandle_t> h(K);
  for (int k = 0; k < K; ++k) CHECK(hipMemCreate(&h[k], S, &prop, 0));
  auto map = [&](int k) {
    void* v = nullptr;
    CHECK(hipMemAddressReserve(&v, S, 4096, nullptr, 0));
    CHECK(hipMemMap(v, S, 0, h[k], 0));
    CHECK(hipMemSetAccess(v, S, &acc, 1));
    return (float*)v;
  };
  float* A = map(0);
  float* A2 = map(0);
  std::vector<float*> B(K), C(K);
  for (int k = 1; k < K; ++k) B[k] = map(k);
  void* gap = nullptr;  // push the second set of mappings far away in VA
  CHECK(hipMemAddressReserve(&gap, 64ull << 30, 4096, nullptr, 0));
  for (int k = 1; k < K; ++k) C[k] = map(k);
  const int per = 4096;
  const unsigned blocks = (unsigned)(S / 16 / per);
  for (int k = 1; k < K; ++k) {
    printf("H_%2d: pair(A,B_k) %5.0f  pair(A,C_k) %5.0f  pair(A2,B_k) %5.0f  pair(A2,C_k) %5.0f GB/s   (B_k %p C_k %p)\n", k,
           timeit(2.0 * S, [&] { hipLaunchKernelGGL(two, dim3(blocks), dim3(256), 0, 0, A, B[k], per); }),
           timeit(2.0 * S, [&] { hipLaunchKernelGGL(two, dim3(blocks), dim3(256), 0, 0, A, C[k], per); }),
           timeit(2.0 * S, [&] { hipLaunchKernelGGL(two, dim3(blocks), dim3(256), 0, 0, A2, B[k], per); }),
           timeit(2.0 * S, [&] { hipLaunchKernelGGL(two, dim3(blocks), dim3(256), 0, 0, A2, C[k], per); }),
           (void*)B[k], (void*)C[k]);
  }
  return 0;  // process exit releases everything (never unmap: the re-map hazard)
}
