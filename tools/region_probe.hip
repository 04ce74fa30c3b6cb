// region_probe.hip — placement map of MI355X HBM for the raster's two write streams.
// Fills the device with 4 GiB hipMalloc chunks (allocation order), then measures
//   single: one 16-B nontemporal store stream over chunk k;
//   pair:   two concurrent streams (chunk 0, chunk k), the raster's newest-only pattern.
// Median of 5 timed launches (GB/s).  Question: is a "fast placement" a property of a region
// of physical memory, or of the pair of regions written together?
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>
#include <functional>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ __launch_bounds__(256) void one(float* __restrict__ a, int per_block) {
  const long base = (long)blockIdx.x * per_block;
  for (int k = threadIdx.x; k < per_block; k += 256) {
    f32x4 x = {(float)k, 1.f, 2.f, 3.f};
    __builtin_nontemporal_store(x, (f32x4*)a + base + k);
  }
}
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
  std::vector<float*> ch;
  for (int k = 0; k < 80; ++k) {
    float* p = nullptr;
    if (hipMalloc(&p, S) != hipSuccess) { (void)hipGetLastError(); break; }
    ch.push_back(p);
  }
  const int per = 4096;
  const unsigned blocks = (unsigned)(S / 16 / per);
  printf("%zu chunks of 4 GiB\n", ch.size());
  for (size_t k = 0; k < ch.size(); ++k) {
    const float s1 = timeit(1.0 * S, [&] { hipLaunchKernelGGL(one, dim3(blocks), dim3(256), 0, 0, ch[k], per); });
    const float p0 = k ? timeit(2.0 * S, [&] { hipLaunchKernelGGL(two, dim3(blocks), dim3(256), 0, 0, ch[0], ch[k], per); }) : 0.f;
    const float pm = k + 1 < ch.size() ? timeit(2.0 * S, [&] { hipLaunchKernelGGL(two, dim3(blocks), dim3(256), 0, 0, ch[k], ch[k + 1], per); }) : 0.f;
    printf("chunk %2zu at %p: single %5.0f   pair(0,k) %5.0f   pair(k,k+1) %5.0f GB/s\n", k, (void*)ch[k], s1, p0, pm);
  }
  for (float* p : ch) CHECK(hipFree(p));
  return 0;
}
