// offset_probe.hip — does the raster's store bandwidth depend on the relative offset of the
// planes it writes concurrently?  (tools/ring_alias_probe: a frame plane in VMM memory plus a
// potential plane from hipMalloc ran 7.1 TB/s, both from hipMalloc or both from VMM 5.8.)
// One hipMalloc buffer; plane A at 0, plane B at S + d (S = plane bytes), for several d; the
// raster's newest-only pattern (2 planes, 16-B nontemporal stores, 4 cells per lane) and its
// full pattern (3 planes: B at S + d, C at 2S + 2d).  Median of 7 launches.
// usage: offset_probe [G=256] [N=32768]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <int P>
__global__ __launch_bounds__(256) void planes(float* __restrict__ a, float* __restrict__ b, float* __restrict__ c,
                                              int G2, int bpe, int cpb) {
  const long e = blockIdx.x / bpe;
  const int tile = blockIdx.x - e * bpe;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int qend = min((tile + 1) * cpb, G2);
  for (int q0 = tile * cpb + wave * 256; q0 < qend; q0 += 1024) {
    const long q = e * (long)G2 + q0 + lane * 4;
    f32x4 x = {(float)q0, 0.f, 1.f, 2.f};
    f32x4 y = {6.f, 7.f, (float)lane, 8.f};
    __builtin_nontemporal_store(x, (f32x4*)(a + q));
    __builtin_nontemporal_store(y, (f32x4*)(b + q));
    if (P == 3) __builtin_nontemporal_store(x + y, (f32x4*)(c + q));
  }
}

template <int P>
static float bw(float* a, float* b, float* c, int G2, long N, int cpb) {
  const int bpe = (G2 + cpb - 1) / cpb;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::vector<float> ms;
  for (int r = 0; r < 8; ++r) {
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(planes<P>, dim3((unsigned)(N * bpe)), dim3(256), 0, 0, a, b, c, G2, bpe, cpb);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float t;
    CHECK(hipEventElapsedTime(&t, e0, e1));
    if (r) ms.push_back(t);
  }
  std::sort(ms.begin(), ms.end());
  return (float)(P * 4.0 * G2 * N / (ms[ms.size() / 2] * 1e-3) / 1e9);
}

int main(int argc, char** argv) {
  const int G = argc > 1 ? atoi(argv[1]) : 256;
  const long N = argc > 2 ? atol(argv[2]) : 32768;
  const int G2 = G * G;
  const size_t S = (size_t)N * G2 * 4;
  const size_t maxd = 9ull << 30;
  char* buf;
  CHECK(hipMalloc(&buf, 2 * S + maxd + (4 << 20)));
  const size_t ds[] = {0, 4096, 1 << 20, 64ull << 20, 256ull << 20, 512ull << 20, 1ull << 30, 1536ull << 20,
                       2ull << 30, 3ull << 30, 4ull << 30, 5ull << 30, 6ull << 30, 7ull << 30, 8ull << 30, 9ull << 30};
  printf("plane %zu B at %p\n", S, (void*)buf);
  for (size_t d : ds) {
    float* a = (float*)buf;
    float* b = (float*)(buf + S + d);
    printf("d=%6.3f GiB  2 planes: cpb4096 %7.1f cpb16384 %7.1f GB/s\n", d / 1073741824.0,
           bw<2>(a, b, b, G2, N, 4096), bw<2>(a, b, b, G2, N, 16384));
  }
  CHECK(hipFree(buf));
  return 0;
}
