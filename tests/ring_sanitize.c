/* The seamless frame ring's host code (ffmp_ring.hip: pieces, pool, reference counts, pairing
 * probes, rebuild, DLPack ownership) driven from plain C on a GPU, for a libffmp whose HOST code
 * is built with AddressSanitizer + UndefinedBehaviorSanitizer (tools/gpu_sanitize.sh; GPU code is
 * not sanitized).  Checks on the way:
 *   - a write through slot 0 is read back through the alias slot W (and the reverse),
 *   - a ring held by a DLPack tensor outlives ffmp_ring_destroy and is parked by the deleter,
 *   - a rebuild shares the kept slots' memory with the old ring and replaces the masked one,
 *   - parked pieces return to the pool and a later ring draws from it.
 * Exit code 0 = all checks passed (the sanitizers abort on their own findings). */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ffmp.h"

#define CHECK(cond)                                                                               \
  do {                                                                                            \
    if (!(cond)) {                                                                                \
      fprintf(stderr, "%s:%d: check failed: %s (last error: %s)\n", __FILE__, __LINE__, #cond, \
              ffmp_last_error());                                                                 \
      return 1;                                                                                   \
    }                                                                                             \
  } while (0)

typedef struct dl_managed {
  struct {
    void* data;
    int32_t device_type, device_id, ndim;
    uint8_t code, bits;
    uint16_t lanes;
    int64_t *shape, *strides;
    uint64_t byte_offset;
  } dl_tensor;
  void* manager_ctx;
  void (*deleter)(struct dl_managed*);
} dl_managed_t;

static int word_at(const void* dev, uint32_t* out) {
  return hipMemcpy(out, dev, sizeof(uint32_t), hipMemcpyDeviceToHost) == hipSuccess;
}

int main(void) {
  const int64_t slot = 256ll << 20;  /* one 256-MiB piece per slot: the pairing probe runs */
  const int W = 3;
  void* partner = NULL;
  CHECK(hipMalloc(&partner, (size_t)slot) == hipSuccess);

  ffmp_ring_t* a = NULL;
  void* base = NULL;
  int64_t stride = 0;
  CHECK(ffmp_ring_create(0, slot, W, partner, slot, &a, &base, &stride) == FFMP_OK);
  CHECK(a != NULL && base != NULL && stride >= slot);
  double info[5];
  CHECK(ffmp_ring_info(a, info, 5) == 5 && info[0] == W && info[2] > 0);
  printf("ring: pieces %.0f fresh %.0f probes %.0f pair GB/s %.0f-%.0f\n", info[0], info[1], info[2], info[3], info[4]);

  /* the alias: slot W maps slot 0's pages */
  char* b = (char*)base;
  uint32_t v = 0;
  CHECK(hipMemset(b, 0x5A, 4096) == hipSuccess);
  CHECK(word_at(b + (size_t)W * stride, &v) && v == 0x5A5A5A5Au);
  CHECK(hipMemset(b + (size_t)W * stride + 64, 0x33, 64) == hipSuccess);
  CHECK(word_at(b + 64, &v) && v == 0x33333333u);
  CHECK(hipMemset(b + stride, 0x11, 4096) == hipSuccess);  /* slot 1 */

  /* a DLPack tensor over the ring keeps it alive past ffmp_ring_destroy */
  const int64_t shape[2] = {W + 1, stride / 4}, strides[2] = {stride / 4, 1};
  dl_managed_t* t = (dl_managed_t*)ffmp_dlpack(base, 2 /* kDLCUDA-like device */, 0, 2, shape, strides, 32, a);
  CHECK(t != NULL);

  /* rebuild slot 1: slots 0 and 2 are shared with `a`, slot 1 is new memory */
  ffmp_ring_t* r = NULL;
  void* rbase = NULL;
  int64_t rstride = 0;
  CHECK(ffmp_ring_rebuild(a, 1u << 1, partner, slot, &r, &rbase, &rstride) == FFMP_OK);
  CHECK(r != NULL && rbase != NULL && rstride == stride && rbase != base);
  CHECK(hipMemset(rbase, 0x77, 4096) == hipSuccess);  /* slot 0 through the new ring */
  CHECK(word_at(b, &v) && v == 0x77777777u);          /* ... is slot 0 of the old one */
  CHECK(word_at(b + (size_t)W * stride, &v) && v == 0x77777777u);
  CHECK(hipMemset((char*)rbase + rstride, 0x22, 4096) == hipSuccess);  /* the replaced slot 1 */
  CHECK(word_at(b + stride, &v) && v == 0x11111111u);                  /* old slot 1 untouched */

  CHECK(ffmp_ring_destroy(a) == FFMP_OK);  /* the tensor still holds `a` */
  CHECK(word_at(b + stride, &v) && v == 0x11111111u);
  t->deleter(t);                           /* last reference: a's own piece (old slot 1) retires */
  CHECK(hipDeviceSynchronize() == hipSuccess);

  /* the next ring draws from the pool once the device is synchronized */
  ffmp_ring_t* c = NULL;
  void* cbase = NULL;
  int64_t cstride = 0;
  CHECK(ffmp_ring_create(0, slot, W, partner, slot, &c, &cbase, &cstride) == FFMP_OK);
  CHECK(ffmp_ring_info(c, info, 5) == 5);
  printf("second ring: pieces %.0f fresh %.0f probes %.0f\n", info[0], info[1], info[2]);
  CHECK(hipMemset(cbase, 0x44, 4096) == hipSuccess);
  CHECK(word_at((char*)cbase + (size_t)W * cstride, &v) && v == 0x44444444u);

  /* compact-layout pairing (partner twice the slot bytes) */
  void* partner2 = NULL;
  CHECK(hipMalloc(&partner2, (size_t)(2 * slot)) == hipSuccess);
  ffmp_ring_t* d = NULL;
  void* dbase = NULL;
  int64_t dstride = 0;
  CHECK(ffmp_ring_create(0, slot, W, partner2, 2 * slot, &d, &dbase, &dstride) == FFMP_OK);
  CHECK(ffmp_ring_info(d, info, 5) == 5 && info[2] > 0);
  printf("compact-pairing ring: probes %.0f pair GB/s %.0f-%.0f\n", info[2], info[3], info[4]);

  CHECK(ffmp_ring_destroy(r) == FFMP_OK);
  CHECK(ffmp_ring_destroy(c) == FFMP_OK);
  CHECK(ffmp_ring_destroy(d) == FFMP_OK);
  CHECK(hipDeviceSynchronize() == hipSuccess);
  CHECK(ffmp_ring_pool_bytes(0) > 0);
  CHECK(hipFree(partner) == hipSuccess && hipFree(partner2) == hipSuccess);
  printf("ring_sanitize ok: pool %lld MiB\n", (long long)(ffmp_ring_pool_bytes(0) >> 20));
  return 0;
}
