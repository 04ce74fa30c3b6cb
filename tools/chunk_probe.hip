// chunk_probe.hip — is store bandwidth a property of physical memory regions?
// Allocates `nchunks` separate 1 GiB buffers (in order), then measures, per chunk, the raster
// store pattern (3 planes of N x G^2 f32, 16-B stores, 4096 cells per block) confined to it.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ __launch_bounds__(256) void three_planes(float* __restrict__ sm, float* __restrict__ pot, int G2, int bpe,
                                                    int cpb) {
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
    *(f32x4*)(m0 + q) = a;
    *(f32x4*)(m1 + q) = a;
    *(f32x4*)(pp + q) = a;
  }
}

int main(int argc, char** argv) {
  const int nchunks = argc > 1 ? atoi(argv[1]) : 200;
  const long chunk = (argc > 2 ? atol(argv[2]) : 1L) << 30;
  const int G = 256;
  const long G2 = (long)G * G;
  const long N = (chunk * 3 / 4) / (3 * G2 * 4);  // 3 planes filling 3/4 of the chunk
  const int cpb = 4096, bpe = (int)(G2 / cpb);
  const double bytes = N * 3.0 * G2 * 4;
  std::vector<char*> bufs;
  for (int c = 0; c < nchunks; ++c) {
    char* p;
    if (hipMalloc(&p, chunk) != hipSuccess) break;
    bufs.push_back(p);
  }
  printf("allocated %zu chunks of %ld GiB (N=%ld envs per chunk)\n", bufs.size(), chunk >> 30, N);
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  std::vector<float> gbs;
  for (size_t c = 0; c < bufs.size(); ++c) {
    float* sm = (float*)bufs[c];
    float* pot = (float*)(bufs[c] + N * 2 * G2 * 4);
    hipLaunchKernelGGL(three_planes, dim3(N * bpe), dim3(256), 0, 0, sm, pot, (int)G2, bpe, cpb);
    CHECK(hipEventRecord(a));
    for (int r = 0; r < 20; ++r) hipLaunchKernelGGL(three_planes, dim3(N * bpe), dim3(256), 0, 0, sm, pot, (int)G2, bpe, cpb);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    ms /= 20;
    gbs.push_back(bytes / ms / 1e6);
  }
  for (size_t c = 0; c < gbs.size(); ++c) printf("%zu:%.0f%s", c, gbs[c], (c % 10 == 9) ? "\n" : " ");
  printf("\n");
  std::vector<float> s = gbs;
  std::sort(s.begin(), s.end());
  printf("min %.0f p25 %.0f median %.0f p75 %.0f max %.0f\n", s[0], s[s.size() / 4], s[s.size() / 2],
         s[3 * s.size() / 4], s.back());
  // whole-footprint run spanning 26 consecutive chunks at a time (like one C3 arena)
  for (auto p : bufs) CHECK(hipFree(p));
  return 0;
}
