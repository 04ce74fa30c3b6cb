// ring_reuse_probe.hip — does a VMM ring mapped where an earlier, unmapped ring lived see its
// first kernel's writes?  (FFMPVec saw the first raster into a fresh seamless ring vanish after
// larger rings had been created and destroyed in the same process.)
// For each teardown variant: create ring A (big, aliased), write it, destroy it; create ring B
// (small, aliased) — usually at a reused address —, one kernel writes a pattern through B, a
// second kernel and a D2H copy check it.
// usage: ring_reuse_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at line %d: %s\n", hipGetErrorString(e), __LINE__, #x); exit(1); } } while (0)

__global__ void fill_pattern(unsigned* p, long n, unsigned salt) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) p[i] = (unsigned)i * 2654435761u ^ salt;
}
__global__ void check_pattern(const unsigned* p, long n, unsigned salt, unsigned long long* bad) {
  unsigned long long b = 0;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) b += (p[i] != ((unsigned)i * 2654435761u ^ salt));
  if (b) atomicAdd(bad, b);
}

struct Ring { char* va; size_t stride, vbytes; int slots; hipMemGenericAllocationHandle_t h0, h1; };

static hipMemAllocationProp prop() {
  hipMemAllocationProp p = {};
  p.type = hipMemAllocationTypePinned;
  p.location.type = hipMemLocationTypeDevice;
  p.location.id = 0;
  return p;
}

static Ring make(size_t stride, int slots, bool alias) {
  Ring r = {};
  hipMemAllocationProp p = prop();
  r.stride = stride; r.slots = slots; r.vbytes = stride * (slots + 1);
  CHECK(hipMemCreate(&r.h0, stride, &p, 0));
  CHECK(hipMemCreate(&r.h1, stride * (slots - 1), &p, 0));
  CHECK(hipMemAddressReserve((void**)&r.va, r.vbytes, 4096, nullptr, 0));
  CHECK(hipMemMap(r.va, stride, 0, r.h0, 0));
  CHECK(hipMemMap(r.va + stride, stride * (slots - 1), 0, r.h1, 0));
  if (alias) CHECK(hipMemMap(r.va + stride * slots, stride, 0, r.h0, 0));
  hipMemAccessDesc acc = {};
  acc.location = p.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  CHECK(hipMemSetAccess(r.va, alias ? r.vbytes : stride * slots, &acc, 1));
  return r;
}

static void destroy(Ring& r, int variant, bool alias) {
  CHECK(hipDeviceSynchronize());
  if (variant == 0) {  // alias, rest, slot 0 (libffmp's order)
    if (alias) CHECK(hipMemUnmap(r.va + r.stride * r.slots, r.stride));
    CHECK(hipMemUnmap(r.va + r.stride, r.stride * (r.slots - 1)));
    CHECK(hipMemUnmap(r.va, r.stride));
  } else if (variant == 1) {  // slot 0, rest, alias
    CHECK(hipMemUnmap(r.va, r.stride));
    CHECK(hipMemUnmap(r.va + r.stride, r.stride * (r.slots - 1)));
    if (alias) CHECK(hipMemUnmap(r.va + r.stride * r.slots, r.stride));
  } else {  // the whole range at once
    CHECK(hipMemUnmap(r.va, alias ? r.vbytes : r.stride * r.slots));
  }
  CHECK(hipMemAddressFree(r.va, r.vbytes));
  CHECK(hipMemRelease(r.h1));
  CHECK(hipMemRelease(r.h0));
  CHECK(hipDeviceSynchronize());
}

static unsigned long long first_write_bad(const Ring& b, unsigned long long* dbad, unsigned salt) {
  const long nw = (long)(b.stride * b.slots / 4);
  CHECK(hipMemset(dbad, 0, 8));
  hipLaunchKernelGGL(fill_pattern, dim3(1024), dim3(256), 0, 0, (unsigned*)b.va, nw, salt);
  hipLaunchKernelGGL(check_pattern, dim3(1024), dim3(256), 0, 0, (const unsigned*)b.va, nw, salt, dbad);
  unsigned long long bad = 0;
  CHECK(hipMemcpy(&bad, dbad, 8, hipMemcpyDeviceToHost));
  std::vector<unsigned> h(nw);
  CHECK(hipMemcpy(h.data(), b.va, nw * 4, hipMemcpyDeviceToHost));
  unsigned long long badh = 0;
  for (long i = 0; i < nw; ++i) badh += h[i] != ((unsigned)i * 2654435761u ^ salt);
  return bad * 1000000000ull + badh;
}

int main() {
  CHECK(hipSetDevice(0));
  unsigned long long* dbad;
  CHECK(hipMalloc(&dbad, 8));
  const size_t big = 512ull << 20, small = 655360;
  for (int alias = 1; alias >= 0; --alias) {
    for (int variant = 0; variant < 3; ++variant) {
      for (int rep = 0; rep < 3; ++rep) {
        Ring a = make(big, 8, alias);
        hipLaunchKernelGGL(fill_pattern, dim3(4096), dim3(256), 0, 0, (unsigned*)a.va, (long)(big * 8 / 4), 7u);
        destroy(a, variant, alias);
        Ring b = make(small, 3, alias);
        unsigned long long r = first_write_bad(b, dbad, 99u + rep);
        printf("alias=%d variant=%d rep=%d  A at %p  B at %p  bad(kernel*1e9 + d2h) = %llu\n", alias, variant, rep,
               (void*)a.va, (void*)b.va, r);
        destroy(b, variant, alias);
      }
    }
  }
  printf("done\n");
  return 0;
}
