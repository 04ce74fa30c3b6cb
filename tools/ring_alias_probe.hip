// ring_alias_probe.hip — can the frame ring be made seamless with HIP virtual memory?
//
// The frame ring (vec_env.py) keeps W slots of N*G^2 float32 and views state_m as slots
// [p, p+1]; when p+1 would run past the last slot it wraps to slot 0 and re-rasters BOTH
// frames (one extra frame every W-1 steps).  If slot W were a second virtual mapping of the
// physical pages of slot 0, the view could always slide by one and every step would write
// only the new frame.  This probe checks, on the box:
//   1. VMM support + granularity;
//   2. aliasing: bytes written (by hipMemset and by a kernel) through the alias of slot 0
//      read back identically through slot 0, and vice versa;
//   3. store bandwidth of the raster's pattern (2 planes of 16-B stores) into VMM-mapped
//      slots vs hipMalloc'd planes of the same size (median of 7 launches, several shapes).
// usage: ring_alias_probe [G=256] [N=32768] [W=8]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at line %d: %s\n", hipGetErrorString(e), __LINE__, #x); exit(1); } } while (0)

__global__ __launch_bounds__(256) void fill_pattern(unsigned* p, long n, unsigned salt) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) p[i] = (unsigned)i * 2654435761u ^ salt;
}

__global__ __launch_bounds__(256) void check_pattern(const unsigned* p, long n, unsigned salt, unsigned long long* bad) {
  unsigned long long b = 0;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) b += (p[i] != ((unsigned)i * 2654435761u ^ salt));
  if (b) atomicAdd(bad, b);
}

// the raster's newest-only store pattern: frame plane + potential plane, 4 cells per lane
__global__ __launch_bounds__(256) void two_planes(float* __restrict__ fr, float* __restrict__ pot, int G2, int bpe, int cpb) {
  const long e = blockIdx.x / bpe;
  const int tile = blockIdx.x - e * bpe;
  float* m = fr + e * (long)G2;
  float* pp = pot + e * (long)G2;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int qend = min((tile + 1) * cpb, G2);
  for (int q0 = tile * cpb + wave * 256; q0 < qend; q0 += 1024) {
    const int q = q0 + lane * 4;
    f32x4 a = {(float)q, 0.f, 1.f, 2.f};
    f32x4 c = {6.f, 7.f, (float)lane, 8.f};
    __builtin_nontemporal_store(a, (f32x4*)(m + q));
    __builtin_nontemporal_store(c, (f32x4*)(pp + q));
  }
}

static float bw(float* fr, float* pot, int G2, long N, int cpb) {
  const int bpe = (G2 + cpb - 1) / cpb;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  std::vector<float> ms;
  for (int r = 0; r < 8; ++r) {
    CHECK(hipEventRecord(a));
    hipLaunchKernelGGL(two_planes, dim3((unsigned)(N * bpe)), dim3(256), 0, 0, fr, pot, G2, bpe, cpb);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float t;
    CHECK(hipEventElapsedTime(&t, a, b));
    if (r) ms.push_back(t);
  }
  std::sort(ms.begin(), ms.end());
  return (float)(2.0 * 4.0 * G2 * N / (ms[ms.size() / 2] * 1e-3) / 1e9);
}

int main(int argc, char** argv) {
  const int G = argc > 1 ? atoi(argv[1]) : 256;
  const long N = argc > 2 ? atol(argv[2]) : 32768;
  const int W = argc > 3 ? atoi(argv[3]) : 8;
  const int G2 = G * G;
  int dev = 0, vmm = 0;
  CHECK(hipSetDevice(dev));
  CHECK(hipDeviceGetAttribute(&vmm, hipDeviceAttributeVirtualMemoryManagementSupported, dev));
  printf("vmm supported: %d\n", vmm);
  if (!vmm) return 0;
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = dev;
  size_t gmin = 0, grec = 0;
  CHECK(hipMemGetAllocationGranularity(&gmin, &prop, hipMemAllocationGranularityMinimum));
  CHECK(hipMemGetAllocationGranularity(&grec, &prop, hipMemAllocationGranularityRecommended));
  const size_t slot = (size_t)N * G2 * 4;
  printf("granularity min %zu rec %zu; slot %zu B (%s multiple)\n", gmin, grec, slot, slot % gmin ? "NOT a" : "a");
  if (slot % gmin) return 0;

  // physical: slot 0 alone, slots 1..W-1 together; virtual: [0 .. W] with slot W = slot 0
  hipMemGenericAllocationHandle_t h0, h1;
  CHECK(hipMemCreate(&h0, slot, &prop, 0));
  CHECK(hipMemCreate(&h1, slot * (W - 1), &prop, 0));
  void* va = nullptr;
  const size_t vbytes = slot * (W + 1);
  CHECK(hipMemAddressReserve(&va, vbytes, grec > gmin ? grec : gmin, nullptr, 0));
  char* base = (char*)va;
  CHECK(hipMemMap(base, slot, 0, h0, 0));
  CHECK(hipMemMap(base + slot, slot * (W - 1), 0, h1, 0));
  hipError_t am = hipMemMap(base + slot * W, slot, 0, h0, 0);
  printf("second mapping of slot 0: %s\n", hipGetErrorString(am));
  if (am != hipSuccess) return 0;
  hipMemAccessDesc acc = {};
  acc.location = prop.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  CHECK(hipMemSetAccess(base, vbytes, &acc, 1));
  printf("mapped %zu B virtual over %zu B physical at %p\n", vbytes, slot * W, va);

  // 2. aliasing, DMA path: memset the alias, copy back through slot 0
  const size_t chk = std::min(slot, (size_t)64 << 20);
  std::vector<unsigned char> host(chk);
  CHECK(hipMemset(base + slot * W, 0xAB, chk));
  CHECK(hipMemcpy(host.data(), base, chk, hipMemcpyDeviceToHost));
  size_t badd = 0;
  for (size_t i = 0; i < chk; ++i) badd += host[i] != 0xAB;
  printf("memset via alias -> read via slot 0: %zu bad bytes of %zu\n", badd, chk);
  // kernel path, whole slot: write through the alias, check through slot 0, then the reverse
  unsigned long long* dbad;
  CHECK(hipMalloc(&dbad, 8));
  const long nw = (long)(slot / 4);
  unsigned long long bad = 0;
  CHECK(hipMemset(dbad, 0, 8));
  hipLaunchKernelGGL(fill_pattern, dim3(8192), dim3(256), 0, 0, (unsigned*)(base + slot * W), nw, 0x1234u);
  hipLaunchKernelGGL(check_pattern, dim3(8192), dim3(256), 0, 0, (const unsigned*)base, nw, 0x1234u, dbad);
  CHECK(hipMemcpy(&bad, dbad, 8, hipMemcpyDeviceToHost));
  printf("kernel write via alias -> kernel read via slot 0: %llu bad words of %ld\n", bad, nw);
  CHECK(hipMemset(dbad, 0, 8));
  hipLaunchKernelGGL(fill_pattern, dim3(8192), dim3(256), 0, 0, (unsigned*)base, nw, 0x9876u);
  hipLaunchKernelGGL(check_pattern, dim3(8192), dim3(256), 0, 0, (const unsigned*)(base + slot * W), nw, 0x9876u, dbad);
  CHECK(hipMemcpy(&bad, dbad, 8, hipMemcpyDeviceToHost));
  printf("kernel write via slot 0 -> kernel read via alias: %llu bad words of %ld\n", bad, nw);
  CHECK(hipDeviceSynchronize());

  // 3. bandwidth: frame slot (VMM) + potential plane (hipMalloc or VMM) vs both hipMalloc
  float* pot;
  float* frm;
  CHECK(hipMalloc(&pot, slot));
  CHECK(hipMalloc(&frm, slot));
  hipMemGenericAllocationHandle_t hp;
  CHECK(hipMemCreate(&hp, slot, &prop, 0));
  void* vpot = nullptr;
  CHECK(hipMemAddressReserve(&vpot, slot, gmin, nullptr, 0));
  CHECK(hipMemMap(vpot, slot, 0, hp, 0));
  CHECK(hipMemSetAccess(vpot, slot, &acc, 1));
  const int shapes[] = {4096, 8192, 16384};
  for (int rep = 0; rep < 2; ++rep)
  for (int cpb : shapes) {
    float vm1 = bw((float*)(base + slot * 3), pot, G2, N, cpb);
    float vmw = bw((float*)(base + slot * W), pot, G2, N, cpb);
    float vv = bw((float*)(base + slot * 3), (float*)vpot, G2, N, cpb);
    float mv = bw(frm, (float*)vpot, G2, N, cpb);
    float mal = bw(frm, pot, G2, N, cpb);
    printf("cpb=%5d  frame VMM slot 3 + pot hipMalloc: %7.1f  alias slot W + pot hipMalloc: %7.1f  "
           "both VMM: %7.1f  frame hipMalloc + pot VMM: %7.1f  both hipMalloc: %7.1f GB/s\n", cpb, vm1, vmw, vv, mv, mal);
  }
  CHECK(hipFree(pot));
  CHECK(hipFree(frm));
  CHECK(hipFree(dbad));
  CHECK(hipMemUnmap(base, slot));
  CHECK(hipMemUnmap(base + slot, slot * (W - 1)));
  CHECK(hipMemUnmap(base + slot * W, slot));
  CHECK(hipMemAddressFree(va, vbytes));
  CHECK(hipMemRelease(h0));
  CHECK(hipMemRelease(h1));
  printf("done\n");
  return 0;
}
