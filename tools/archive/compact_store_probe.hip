// compact_store_probe.hip — store-pattern ceilings of the compact layout (uint8 frame + binary16
// potential, FFMP_OBS_U8F16) at C3 size (32,768 planes of 256 x 256), no cell arithmetic:
//   ct4     the current CT4 tiles: a wave task is 4 rows x 64 columns, a lane 4 cells = one 4-B
//           frame store + one 8-B potential store (waves of a block on neighbouring column bands)
//   ct4x4   4 such tasks per wave gathered into 16 rows x 64 columns, stored as 16 B per lane
//           (frame: one store, 4 lanes per row; potential: two stores, 8 lanes per row)
//   rows    a wave task is whole rows: 16-B lane stores, 1 KiB contiguous per instruction
//   ct4lds  ct4 tiles staged through LDS per 16 rows x 256 columns, stored as whole rows
//   f32     the float32 layout's CT4-shaped tile (16-B frame + 16-B potential per lane), for scale
// Each pattern writes every byte of both planes once per launch; median of 7 launches (GB/s).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <vector>
#include <algorithm>
#include <functional>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int G = 256, G2 = G * G;

// one block per plane (65,536 cells), 4 waves
template <int PAT>
__global__ __launch_bounds__(256) void probe(uint8_t* __restrict__ fr, uint16_t* __restrict__ pot, float* __restrict__ f32a,
                                             float* __restrict__ f32b, int n) {
  const int e = blockIdx.x;
  if (e >= n) return;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint8_t* b = fr + (int64_t)e * G2;
  uint16_t* h = pot + (int64_t)e * G2;
  const uint32_t v = 0x01010101u * (uint32_t)(e & 0xFF);
  if (PAT == 0) {  // ct4: column band = wave, 64 bands of 4 rows
    const int r = lane >> 4, cl = (lane & 15) * 4, j = wave * 64 + cl;
    for (int band = 0; band < G / 4; ++band) {
      const int q = (band * 4 + r) * G + j;
      __builtin_nontemporal_store(v + band, reinterpret_cast<uint32_t*>(b + q));
      u32x2 p = {v, v + band};
      __builtin_nontemporal_store(p, reinterpret_cast<u32x2*>(h + q));
    }
  } else if (PAT == 1) {  // ct4x4: 16 rows x 64 columns per group of 4 tasks
    const int j = wave * 64;
    for (int grp = 0; grp < G / 16; ++grp) {
      const int rf = grp * 16 + (lane >> 2), cf = j + (lane & 3) * 16;
      u32x4 w = {v, v + 1, v + 2, v + grp};
      __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(b + rf * G + cf));
      const int rp = grp * 16 + (lane >> 3), cp = j + (lane & 7) * 8;
      __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(h + rp * G + cp));
      __builtin_nontemporal_store(w + 1u, reinterpret_cast<u32x4*>(h + (rp + 8) * G + cp));
    }
  } else if (PAT == 2) {  // rows: wave w owns rows w, w+4, ...; 16-B lane stores
    for (int q0 = wave * 1024; q0 < G2; q0 += 4096) {
      u32x4 w = {v, v + 1, v + 2, v + (uint32_t)q0};
      __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(b + q0 + lane * 16));
      __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(h + q0 + lane * 8));
      __builtin_nontemporal_store(w + 1u, reinterpret_cast<u32x4*>(h + q0 + 512 + lane * 8));
    }
  } else if (PAT == 4) {  // ct4 tiles computed, staged in LDS per 16 rows, stored as whole rows
    __shared__ uint32_t sf[16 * G / 4];
    __shared__ u32x2 sp[16 * G / 4];
    const int r = lane >> 4, cl = (lane & 15) * 4, j = wave * 64 + cl;
    for (int grp = 0; grp < G / 16; ++grp) {
#pragma unroll
      for (int bb = 0; bb < 4; ++bb) {
        const int row = bb * 4 + r;
        sf[(row * G + j) >> 2] = v + bb;
        u32x2 p = {v, v + (uint32_t)bb};
        sp[(row * G + j) >> 2] = p;
      }
      __syncthreads();
      const u32x4 w = reinterpret_cast<const u32x4*>(sf)[wave * 64 + lane];
      const u32x4 p0 = reinterpret_cast<const u32x4*>(sp)[wave * 128 + lane];
      const u32x4 p1 = reinterpret_cast<const u32x4*>(sp)[wave * 128 + 64 + lane];
      const int64_t q0 = (int64_t)(grp * 16 + wave * 4) * G;
      __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(b + q0) + lane);
      __builtin_nontemporal_store(p0, reinterpret_cast<u32x4*>(h + q0) + lane);
      __builtin_nontemporal_store(p1, reinterpret_cast<u32x4*>(h + q0) + 64 + lane);
      __syncthreads();
    }
  } else {  // f32 ct4 tile (frame + potential, 16 B each per lane)
    float* fa = f32a + (int64_t)e * G2;
    float* fb = f32b + (int64_t)e * G2;
    const int r = lane >> 4, cl = (lane & 15) * 4, j = wave * 64 + cl;
    for (int band = 0; band < G / 4; ++band) {
      const int q = (band * 4 + r) * G + j;
      f32x4 x = {(float)band, 1.f, 2.f, 3.f};
      __builtin_nontemporal_store(x, reinterpret_cast<f32x4*>(fa + q));
      __builtin_nontemporal_store(x + 1.f, reinterpret_cast<f32x4*>(fb + q));
    }
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

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 32768;
  const int rounds = argc > 2 ? atoi(argv[2]) : 3;
  uint8_t* fr;
  uint16_t* pot;
  float *fa, *fb;
  CHECK(hipMalloc(&fr, (size_t)n * G2));
  CHECK(hipMalloc(&pot, (size_t)n * G2 * 2));
  CHECK(hipMalloc(&fa, (size_t)n * G2 * 4));
  CHECK(hipMalloc(&fb, (size_t)n * G2 * 4));
  const double cb = (double)n * G2 * 3, fbytes = (double)n * G2 * 8;
  for (int k = 0; k < rounds; ++k) {
    const float a = timeit(cb, [&] { probe<0><<<n, 256>>>(fr, pot, fa, fb, n); });
    const float b = timeit(cb, [&] { probe<1><<<n, 256>>>(fr, pot, fa, fb, n); });
    const float c = timeit(cb, [&] { probe<2><<<n, 256>>>(fr, pot, fa, fb, n); });
    const float s4 = timeit(cb, [&] { probe<4><<<n, 256>>>(fr, pot, fa, fb, n); });
    const float d = timeit(fbytes, [&] { probe<3><<<n, 256>>>(fr, pot, fa, fb, n); });
    CHECK(hipGetLastError());
    printf("round %d  n=%d  ct4 %.0f  ct4x4 %.0f  rows %.0f  ct4-lds-rows %.0f  f32-ct4 %.0f GB/s\n", k, n, a, b, c, s4, d);
    fflush(stdout);
  }
  CHECK(hipDeviceSynchronize());
  return 0;
}
