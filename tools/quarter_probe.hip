// quarter_probe.hip (derived from placement_probe.hip) — does the store bandwidth of the raster pattern depend on where the
// potential plane sits relative to state_m?  One allocation holds state_m (N x 2 x G^2 f32)
// followed by `pad` bytes and the potential plane (N x G^2 f32); the kernel is the raster's
// pure store pattern (3 x 16-B stores per lane per 1024-cell pass, 4096 cells per block).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <functional>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ __launch_bounds__(256) void three_planes(float* __restrict__ sm, float* __restrict__ pot, int G2, int bpe,
                                                    int cpb, long env_stride_sm, long plane_off) {
  const long e = blockIdx.x / bpe;
  const int tile = blockIdx.x - e * bpe;
  float* m0 = sm + e * env_stride_sm;
  float* m1 = m0 + plane_off;
  float* pp = pot + e * (long)G2;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int qend = min((tile + 1) * cpb, G2);
  for (int q0 = tile * cpb + wave * 256; q0 < qend; q0 += 1024) {
    const int q = q0 + lane * 4;
    f32x4 a = {(float)q, 0.f, 1.f, 2.f};
    *(f32x4*)(m0 + q) = a;
    *(f32x4*)(m1 + q) = a;
    *(f32x4*)(pp + q) = a;
  }
}

static float time_it(std::function<void()> f) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  std::vector<float> ts;
  f();
  CHECK(hipDeviceSynchronize());
  for (int r = 0; r < 7; ++r) {
    CHECK(hipEventRecord(a));
    f();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    ts.push_back(ms);
  }
  std::sort(ts.begin(), ts.end());
  return ts[3];
}

int main(int argc, char** argv) {
  const int G = 256;
  const long N = 32768;
  const long G2 = (long)G * G;
  const int cpb = 4096, bpe = (int)((G2 + cpb - 1) / cpb);
  const long smbytes = N * 2 * G2 * 4;
  const int allocs = argc > 1 ? atoi(argv[1]) : 6;
  for (int r = 0; r < allocs; ++r) {
    char *junk, *buf;
    CHECK(hipMalloc(&junk, (size_t)(r * 53 + 1) << 20));
    CHECK(hipMalloc(&buf, smbytes + N * G2 * 4));
    float* sm = (float*)buf;
    float* pot = (float*)(buf + smbytes);
    const double bytes = N * 3.0 * G2 * 4;
    float t = time_it([&] {
      hipLaunchKernelGGL(three_planes, dim3(N * bpe), dim3(256), 0, 0, sm, pot, (int)G2, bpe, cpb, 2 * G2, G2);
    });
    printf("alloc %d full: %.0f GB/s | quarters:", r, bytes / t / 1e6);
    for (int qd = 0; qd < 4; ++qd) {
      const long n4 = N / 4, e0 = qd * n4;
      float tq = time_it([&] {
        hipLaunchKernelGGL(three_planes, dim3(n4 * bpe), dim3(256), 0, 0, sm + e0 * 2 * G2, pot + e0 * G2, (int)G2, bpe,
                           cpb, 2 * G2, G2);
      });
      printf(" %.0f", n4 * 3.0 * G2 * 4 / tq / 1e6);
    }
    // state_m planes only vs potential only (whole N)
    float ts = time_it([&] {
      hipLaunchKernelGGL(three_planes, dim3(N * bpe), dim3(256), 0, 0, sm, sm + G2, (int)G2, bpe, cpb, 2 * G2, G2);
    });
    printf(" | pot->m1 alias (2 streams) %.0f\n", N * 2.0 * G2 * 4 / ts / 1e6);
    CHECK(hipFree(buf));
    CHECK(hipFree(junk));
  }
  return 0;
}
