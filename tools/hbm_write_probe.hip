// hbm_write_probe.hip — ceiling of the raster kernel's store pattern on MI355X.
// Writes 3 planes of N x G^2 float32 (the state_m pair + potential) with 16-B
// stores, 256-thread blocks, 4 cells per lane per pass, like raster_kernel,
// with plain vs nontemporal stores and several cells-per-block; also a single
// flat stream.  Prints GB/s per variant (hipEvent timing, median of 10).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>
#include <functional>

typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <bool NT>
__global__ __launch_bounds__(256) void three_planes(float* __restrict__ sm, float* __restrict__ pot, int G2, int bpe, int cpb) {
  const long e = blockIdx.x / bpe;
  const int tile = blockIdx.x - e * bpe;
  float* m0 = sm + e * 2L * G2;
  float* m1 = m0 + G2;
  float* pp = pot + e * (long)G2;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int qend = min((tile + 1) * cpb, G2);
  for (int q0 = tile * cpb + wave * 256; q0 < qend; q0 += 1024) {
    const int q = q0 + lane * 4;
    f32x4 a = {(float)q, 0.f, 1.f, 2.f};
    f32x4 b = {3.f, (float)e, 4.f, 5.f};
    f32x4 c = {6.f, 7.f, (float)lane, 8.f};
    if (NT) {
      __builtin_nontemporal_store(a, (f32x4*)(m0 + q));
      __builtin_nontemporal_store(b, (f32x4*)(m1 + q));
      __builtin_nontemporal_store(c, (f32x4*)(pp + q));
    } else {
      *(f32x4*)(m0 + q) = a;
      *(f32x4*)(m1 + q) = b;
      *(f32x4*)(pp + q) = c;
    }
  }
}

// P planes, each lane writes V consecutive float4 per plane per pass (V*16 B per lane).
template <int P, int V, int BS>
__global__ __launch_bounds__(BS) void multi_planes(float* __restrict__ base, long plane_stride, int G2, int bpe, int cpb) {
  const long e = blockIdx.x / bpe;
  const int tile = blockIdx.x - e * bpe;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int qend = min((tile + 1) * cpb, G2);
  constexpr int WAVES = BS / 64;
  for (int q0 = tile * cpb + wave * 256 * V; q0 < qend; q0 += WAVES * 256 * V) {
#pragma unroll
    for (int p = 0; p < P; ++p) {
      float* dst = base + (long)p * plane_stride + e * (long)G2;
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const int q = q0 + (v * 64 + lane) * 4;
        f32x4 a = {(float)q, (float)p, 1.f, 2.f};
        *(f32x4*)(dst + q) = a;
      }
    }
  }
}

template <bool NT>
__global__ __launch_bounds__(256) void flat(float* __restrict__ p, long n4) {
  long i = (long)blockIdx.x * 256 + threadIdx.x;
  const long stride = (long)gridDim.x * 256;
  for (; i < n4; i += stride) {
    f32x4 a = {(float)i, 0.f, 1.f, 2.f};
    if (NT) __builtin_nontemporal_store(a, (f32x4*)p + i);
    else ((f32x4*)p)[i] = a;
  }
}

static float time_it(std::function<void()> f) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  std::vector<float> ts;
  f(); hipDeviceSynchronize();
  for (int r = 0; r < 10; ++r) {
    hipEventRecord(a); f(); hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b); ts.push_back(ms);
  }
  std::sort(ts.begin(), ts.end());
  return ts[5];
}

int main(int argc, char** argv) {
  const int G = argc > 1 ? atoi(argv[1]) : 256;
  const long N = argc > 2 ? atol(argv[2]) : 32768;
  const int G2 = G * G;
  float *sm, *pot;
  CHECK(hipMalloc(&sm, N * 2L * G2 * 4));
  CHECK(hipMalloc(&pot, N * (long)G2 * 4));
  const double bytes = N * 3.0 * G2 * 4;
  for (int cpb : {4096, 8192, 16384, 65536}) {
    if (cpb > G2) continue;
    const int bpe = (G2 + cpb - 1) / cpb;
    const long blocks = N * bpe;
    float t0 = time_it([&] { hipLaunchKernelGGL(three_planes<false>, dim3(blocks), dim3(256), 0, 0, sm, pot, G2, bpe, cpb); });
    float t1 = time_it([&] { hipLaunchKernelGGL(three_planes<true>, dim3(blocks), dim3(256), 0, 0, sm, pot, G2, bpe, cpb); });
    printf("three_planes G=%d N=%ld cpb=%d: plain %.3f ms %.0f GB/s | nt %.3f ms %.0f GB/s\n", G, N, cpb, t0,
           bytes / t0 / 1e6, t1, bytes / t1 / 1e6);
  }
  const long n4 = N * 2L * G2 / 4;
  for (int grid : {2048, 8192, 65536}) {
    float t0 = time_it([&] { hipLaunchKernelGGL(flat<false>, dim3(grid), dim3(256), 0, 0, sm, n4); });
    float t1 = time_it([&] { hipLaunchKernelGGL(flat<true>, dim3(grid), dim3(256), 0, 0, sm, n4); });
    printf("flat grid=%d %.2f GB: plain %.0f GB/s | nt %.0f GB/s\n", grid, n4 * 16 / 1e9, n4 * 16 / t0 / 1e6,
           n4 * 16 / t1 / 1e6);
  }
  // vendor fill as a reference point
  {
    const size_t n32 = N * 2L * G2;
    float t = time_it([&] { (void)hipMemsetD32Async((hipDeviceptr_t)sm, 0x3f800000, n32, 0); });
    printf("hipMemsetD32Async %.2f GB: %.0f GB/s\n", n32 * 4 / 1e9, n32 * 4 / t / 1e6);
  }
  // plane-count / width / block-size variants on the same 3*N*G2 floats (as P planes of N*G2*3/P)
  {
    float* base = sm;  // reuse: sm has 2*N*G2, pot N*G2; treat as one 3*N*G2 region (contiguous? no) -> use sm only
    (void)base;
  }
  {
    float* big;
    CHECK(hipMalloc(&big, N * 3L * G2 * 4));
    const long ps = N * (long)G2;
    auto run = [&](const char* name, auto kern, int P, int V, int BS) {
      const int cpb = 4096;
      const int bpe = (G2 + cpb - 1) / cpb;
      const long planes_env = N * (long)bpe;
      const long stride = ps * 3 / P;   // P planes of equal size covering the same bytes
      const int G2eff = (int)(stride / N);
      const int bpe2 = (G2eff + cpb - 1) / cpb;
      (void)planes_env;
      float t = time_it([&] { hipLaunchKernelGGL(kern, dim3(N * bpe2), dim3(BS), 0, 0, big, stride, G2eff, bpe2, cpb); });
      printf("%-28s P=%d V=%d BS=%d: %.3f ms %.0f GB/s\n", name, P, V, BS, t, bytes / t / 1e6);
    };
    run("multi", multi_planes<3, 1, 256>, 3, 1, 256);
    run("multi", multi_planes<3, 2, 256>, 3, 2, 256);
    run("multi", multi_planes<3, 4, 256>, 3, 4, 256);
    run("multi", multi_planes<3, 1, 512>, 3, 1, 512);
    run("multi", multi_planes<3, 1, 1024>, 3, 1, 1024);
    run("multi", multi_planes<1, 1, 256>, 1, 1, 256);
    run("multi", multi_planes<1, 4, 256>, 1, 4, 256);
    run("multi", multi_planes<6, 1, 256>, 6, 1, 256);
    run("multi", multi_planes<12, 1, 256>, 12, 1, 256);
    CHECK(hipFree(big));
  }
  CHECK(hipFree(sm));
  CHECK(hipFree(pot));
  return 0;
}
