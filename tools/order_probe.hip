// order_probe.hip — raster store pattern under different block->(env, tile) orders, all on
// the SAME allocation, repeated over several fresh allocations.  Tests whether de-correlating
// the in-plane offsets that concurrently running blocks write removes the slow placement mode.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

// MODE 0: env-major (raster_kernel today): e = b / bpe, tile = b % bpe
// MODE 1: env-major, tile rotated by env: tile = (b % bpe + e) % bpe
// MODE 2: tile-major: tile = b / N, e = b % N
// MODE 3: env-major, pass order rotated per block (start pass = e % passes)
// MODE 4: env-major, tile rotated by 5*e and pass rotated
// MODE 5: XCD-aware: block b runs logical block (b % 8) * (nb / 8) + b / 8, so each XCD
//         (blocks b = x mod 8) walks its own contiguous eighth of the envs
template <int MODE>
__global__ __launch_bounds__(256) void three_planes(float* __restrict__ sm, float* __restrict__ pot, int G2, int bpe,
                                                    int cpb, long N) {
  long e;
  int tile;
  if (MODE == 5) {
    const long nb = N * (long)bpe;
    const long b = blockIdx.x;
    const long per = nb / 8;
    const long lb = (b % 8) * per + b / 8;
    e = lb / bpe;
    tile = (int)(lb - e * bpe);
  } else if (MODE == 2) {
    tile = (int)(blockIdx.x / N);
    e = blockIdx.x - (long)tile * N;
  } else {
    e = blockIdx.x / bpe;
    tile = (int)(blockIdx.x - e * bpe);
    if (MODE == 1) tile = (int)((tile + e) % bpe);
    if (MODE == 4) tile = (int)((tile + 5 * e) % bpe);
  }
  float* m0 = sm + e * 2L * G2;
  float* m1 = m0 + G2;
  float* pp = pot + e * (long)G2;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int passes = cpb / 1024;
  const int rot = (MODE == 3 || MODE == 4) ? (int)(e % passes) : 0;
  for (int k = 0; k < passes; ++k) {
    const int p = (k + rot) % passes;
    const int q = tile * cpb + p * 1024 + wave * 256 + lane * 4;
    if (q >= G2) continue;
    f32x4 a = {(float)q, 0.f, 1.f, 2.f};
    *(f32x4*)(m0 + q) = a;
    *(f32x4*)(m1 + q) = a;
    *(f32x4*)(pp + q) = a;
  }
}

template <int MODE>
float run(float* sm, float* pot, int G2, int bpe, int cpb, long N) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL(three_planes<MODE>, dim3(N * bpe), dim3(256), 0, 0, sm, pot, G2, bpe, cpb, N);
  CHECK(hipEventRecord(a));
  for (int r = 0; r < 5; ++r)
    hipLaunchKernelGGL(three_planes<MODE>, dim3(N * bpe), dim3(256), 0, 0, sm, pot, G2, bpe, cpb, N);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
  return ms / 5;
}

int main(int argc, char** argv) {
  const int G = argc > 1 ? atoi(argv[1]) : 256;
  const long N = argc > 2 ? atol(argv[2]) : 32768;
  const int allocs = argc > 3 ? atoi(argv[3]) : 6;
  const int cpb = argc > 4 ? atoi(argv[4]) : 4096;
  const int G2 = G * G, bpe = (G2 + cpb - 1) / cpb;
  const double bytes = N * 3.0 * G2 * 4;
  printf("G=%d N=%ld  GB/s: env-major cpb=%d | xcd-aware cpb=%d | env-major cpb=1024 | xcd-aware cpb=1024 | env-major cpb=16384\n",
         G, N, cpb, cpb);
  for (int r = 0; r < allocs; ++r) {
    float *sm, *pot, *junk;
    CHECK(hipMalloc(&junk, (size_t)(r * 37 + 1) << 20));
    CHECK(hipMalloc(&sm, N * 2L * G2 * 4));
    CHECK(hipMalloc(&pot, N * (long)G2 * 4));
    const int bpe1 = (G2 + 1023) / 1024, bpe16 = (G2 + 16383) / 16384;
    float t[5];
    t[0] = run<0>(sm, pot, G2, bpe, cpb, N);
    t[1] = run<5>(sm, pot, G2, bpe, cpb, N);
    t[2] = run<0>(sm, pot, G2, bpe1, 1024, N);
    t[3] = run<5>(sm, pot, G2, bpe1, 1024, N);
    t[4] = run<0>(sm, pot, G2, bpe16, 16384, N);
    printf("alloc %d: %.0f | %.0f | %.0f | %.0f | %.0f\n", r, bytes / t[0] / 1e6, bytes / t[1] / 1e6,
           bytes / t[2] / 1e6, bytes / t[3] / 1e6, bytes / t[4] / 1e6);
    CHECK(hipFree(pot));
    CHECK(hipFree(sm));
    CHECK(hipFree(junk));
  }
  return 0;
}
