// ffmp_ring.hip — the seamless frame ring of libffmp (include/ffmp.h ffmp_ring_*, ffmp_dlpack):
// HIP virtual memory for the in-place temporal stack of make_temporal_maps
// (src/train.py:474-486), built from physical pieces paired with the potential plane.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>
#include <atomic>
#include <memory>
#include <mutex>
#include <vector>

#include "ffmp.h"

namespace ffmp_detail {
int fail(int code, const char* fmt, ...);  // ffmp_kernels.hip (sets ffmp_last_error())

// FFMP_TUNE_RING_EXTRA: fresh pieces beyond need per create / rebuild (0 = default, v = cap v - 1)
std::atomic<int32_t> g_ring_extra{0};
// bytes of virtual address space reserved so far per device (never freed: see ffmp_ring_va_reserved)
constexpr int kVaDevices = 64;
std::atomic<int64_t> g_va_reserved[kVaDevices];
void note_va(int32_t device, size_t bytes) {
  if (device >= 0 && device < kVaDevices) g_va_reserved[device].fetch_add((int64_t)bytes);
}
int32_t ring_extra_swap(int32_t v) { return g_ring_extra.exchange(v); }
}
using ffmp_detail::fail;

typedef float f32x4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------ seamless frame ring
// Built from physical PIECES (hipMemCreate handles of piece_bytes): slot i of the ring is n
// pieces mapped back to back, and virtual slot W maps slot 0's pieces a second time (the
// alias).  Two findings on MI355X / ROCm 7.2 shape it:
//
// * Pairing.  The raster writes a frame slot and the potential plane in lockstep (same offset,
//   same time).  Two lockstep store streams run at ~6.9 TB/s or at 4.6-5.6 TB/s depending on
//   the PHYSICAL memory each lands in (tools/pair_alias_probe.hip: two virtual mappings of the
//   same pages pair identically; tools/region_probe.hip), so one slot that pairs badly with
//   the potential plane makes one step in W ~25 % slower.  With a `partner` (the potential
//   plane), every piece position (slot i, piece j) gets a piece measured to pair well with the
//   partner's bytes the raster writes beside it — [j*P, (j+1)*P) in the float32 layout,
//   [2j*P, 2(j+1)*P) for compact uint8 frames beside a binary16 plane (the ratio of partner
//   bytes to slot bytes, RingGeom::scale) — by a two-stream store probe of the same byte ratio,
//   candidates from the free-piece
//   pool first, then fresh pieces; pieces that pair badly here stay pooled for other positions
//   or later rings.
// * Never reuse an address.  Once a VMM range is unmapped and its address reused by a new
//   mapping, the runtime can still resolve the address to the OLD allocation
//   (tools/ring_reuse_probe.hip: D2H copies of a fresh mapping return the previous ring's bytes;
//   FFMPVec saw the first raster into a fresh ring vanish).  So no reservation is ever freed:
//   every piece keeps a private "home" mapping, a ring maps its pieces once more at a fresh
//   address, and a ring whose last reference is dropped returns its pieces to the pool (its
//   addresses are simply never used again).  A pooled piece's physical memory can still be given
//   back (ffmp_ring_pool_trim): every mapping of it (home and the dead rings') is unmapped and the
//   handle released, while the address ranges stay reserved — no later mapping can land there.
// * Sharing.  A piece may sit in several rings at once: ffmp_ring_rebuild leaves `old` whole
//   and maps its kept pieces into the new ring too, so that a caller can time both and keep
//   the faster.  Each piece carries a count of the rings holding it; it is retired when the
//   last one goes.
// * Retired pieces are not reused at once: the DLPack deleter can drop a ring while kernels
//   still write it.  They wait in g_retired until the next ffmp_ring_create / rebuild on that
//   device, which synchronizes the device before drawing from the pool.
struct ffmp_piece {
  hipMemGenericAllocationHandle_t h;
  char* home;  // private mapping, for the pairing probe
  size_t bytes;
  int32_t device;
  int* rings;  // rings holding the piece (shared by every copy; under g_pool_mu)
  std::vector<char*>* maps;  // every address it is mapped at: home, then each ring's (shared; under g_pool_mu)
};

struct ffmp_ring {
  int32_t device;
  int32_t slots;
  size_t stride;  // slot stride = pieces_per_slot * piece bytes
  char* va;
  size_t vbytes;
  int refs;  // the creator + one per live DLPack tensor (atomic)
  std::vector<ffmp_piece> pieces;  // slot-major, slots * pieces_per_slot
  double pair_gbs_min, pair_gbs_max;  // pairing probe of the chosen pieces (0 without partner)
  int pieces_new, pieces_tested;
  int scale;  // partner bytes per slot byte, fixed at create (RingGeom::scale; a rebuild reuses it)
};

// dlpack.h (v0.8) DLManagedTensor, the interchange torch.utils.dlpack.from_dlpack consumes
struct DLDevice_ { int32_t device_type, device_id; };
struct DLDataType_ { uint8_t code, bits; uint16_t lanes; };
struct DLTensor_ {
  void* data;
  DLDevice_ device;
  int32_t ndim;
  DLDataType_ dtype;
  int64_t* shape;
  int64_t* strides;
  uint64_t byte_offset;
};
struct DLManagedTensor_ {
  DLTensor_ dl_tensor;
  void* manager_ctx;
  void (*deleter)(DLManagedTensor_*);
};
struct DLHolder_ {  // one allocation: the managed tensor, its shape/strides, its owner
  DLManagedTensor_ mt;
  int64_t dims[16];
  ffmp_ring* owner;
};

// two lockstep 16-B nontemporal store streams, n16 float4s to `a` and SCALE x n16 to `b`: the
// raster's write pattern (float32 layout: frame and potential plane at the same rate, SCALE 1;
// compact layout: 1-byte frame cells beside 2-byte potential cells, SCALE 2)
// (every store instruction of a wave covers 1 KiB of contiguous bytes of its stream).  n16 need
// not be a multiple of 256 (the last piece beside a compact plane whose size is not): each stream
// is bounded by its own length, n16 float4s of `a` and SCALE x n16 of `b`.
template <int SCALE>
__global__ __launch_bounds__(256) void pair_probe_kernel(f32x4* __restrict__ a, f32x4* __restrict__ b, int64_t n16) {
  const int64_t blk0 = (int64_t)blockIdx.x * 4096;
  const f32x4 x = {0.f, 1.f, 2.f, 3.f};
  for (int k = 0; k < 16; ++k) {
    const int64_t i = blk0 + threadIdx.x + 256 * k;
    if (i >= n16) break;
    __builtin_nontemporal_store(x, a + i);
#pragma unroll
    for (int s = 0; s < SCALE; ++s) {
      const int64_t j = SCALE * blk0 + threadIdx.x + 256 * (SCALE * k + s);
      if (j < SCALE * n16) __builtin_nontemporal_store(x, b + j);
    }
  }
}

namespace {

std::mutex g_pool_mu;
std::vector<ffmp_piece> g_pieces;   // free pieces (mapped at home), reusable
std::vector<ffmp_piece> g_retired;  // free, but GPU work issued before their ring died may still write them

// Best pairing probe seen per (device, partner plane, scale) (choose_pieces' early-accept bar).
// Keyed by the partner: a rebuild against the same plane is judged on the same scale, while a
// relocated plane (FFMPVec._relocate_partner) or another instance starts its own reference, so one
// high probe against some other plane cannot raise every later ring's bar.  Under g_pool_mu.
struct PairRef { int32_t device; int scale; const void* partner; double gbs; };
std::vector<PairRef> g_pair_ref;

double pair_ref_get(int32_t device, int scale, const void* partner) {
  std::lock_guard<std::mutex> lk(g_pool_mu);
  for (const PairRef& p : g_pair_ref)
    if (p.device == device && p.scale == scale && p.partner == partner) return p.gbs;
  return 0.0;
}

void pair_ref_put(int32_t device, int scale, const void* partner, double gbs) {
  std::lock_guard<std::mutex> lk(g_pool_mu);
  for (PairRef& p : g_pair_ref)
    if (p.device == device && p.scale == scale && p.partner == partner) {
      p.gbs = std::max(p.gbs, gbs);
      return;
    }
  if (g_pair_ref.size() >= 256) g_pair_ref.erase(g_pair_ref.begin());  // bounded: oldest planes first
  g_pair_ref.push_back({device, scale, partner, gbs});
}

hipMemAllocationProp dev_prop(int32_t device) {
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = device;
  return prop;
}

hipError_t map_rw(char* va, size_t bytes, hipMemGenericAllocationHandle_t h, int32_t device) {
  hipError_t e = hipMemMap(va, bytes, 0, h, 0);
  if (e != hipSuccess) return e;
  hipMemAccessDesc acc = {};
  acc.location = dev_prop(device).location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  return hipMemSetAccess(va, bytes, &acc, 1);
}

// reservation alignment for pieces of `bytes`: the largest power of two <= min(bytes, 1 GiB),
// at least the granularity (so every piece can map with the largest page fragments)
size_t va_align(size_t bytes, size_t gran) {
  size_t a = gran;
  while (a * 2 <= bytes && a * 2 <= ((size_t)1 << 30)) a *= 2;
  return a;
}

// a fresh piece mapped at its home address; on failure no memory stays allocated (only the
// address reservation of a failed mapping, see below)
hipError_t new_piece(int32_t device, size_t bytes, size_t gran, ffmp_piece* out) {
  hipMemAllocationProp prop = dev_prop(device);
  ffmp_piece p = {};
  p.bytes = bytes;
  p.device = device;
  hipError_t e = hipMemCreate(&p.h, bytes, &prop, 0);
  if (e != hipSuccess) return e;
  if ((e = hipMemAddressReserve((void**)&p.home, bytes, va_align(bytes, gran), nullptr, 0)) != hipSuccess) {
    (void)hipMemRelease(p.h);  // never mapped: safe to give back
    return e;
  }
  ffmp_detail::note_va(device, bytes);
  if ((e = map_rw(p.home, bytes, p.h, device)) != hipSuccess) {
    // The reservation is kept (never freed): an address range that was mapped once must not be
    // handed out again, or the runtime can resolve later accesses there to this allocation.
    (void)hipMemUnmap(p.home, bytes);
    (void)hipMemRelease(p.h);
    return e;
  }
  p.rings = new int(0);  // freed with the piece (ffmp_ring_pool_trim) or never
  p.maps = new std::vector<char*>(1, p.home);
  *out = p;
  return hipSuccess;
}

// GB/s of the two-stream store probe over `bytes` of piece home + scale x `bytes` of partner
// (< 0: the probe did not complete)
double pair_gbs(char* a, char* b, size_t bytes, int scale, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
  const int64_t n16 = (int64_t)(bytes / 16);
  const unsigned blocks = (unsigned)((n16 + 4095) / 4096);
  float best = 1e30f;
  for (int r = 0; r < 4; ++r) {
    (void)hipEventRecord(e0, s);
    if (scale == 2)
      hipLaunchKernelGGL(pair_probe_kernel<2>, dim3(blocks), dim3(256), 0, s, (f32x4*)a, (f32x4*)b, n16);
    else
      hipLaunchKernelGGL(pair_probe_kernel<1>, dim3(blocks), dim3(256), 0, s, (f32x4*)a, (f32x4*)b, n16);
    (void)hipEventRecord(e1, s);
    if (hipEventSynchronize(e1) != hipSuccess) return -1.0;  // a fault: the caller fails loudly
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (r > 0 && ms < best) best = ms;  // first launch warms up
  }
  return (1.0 + scale) * (double)(n16 * 16) / (best * 1e-3) / 1e9;
}

void ring_unref(ffmp_ring* r) {
  if (__atomic_sub_fetch(&r->refs, 1, __ATOMIC_ACQ_REL) > 0) return;
  std::lock_guard<std::mutex> lk(g_pool_mu);
  for (const ffmp_piece& p : r->pieces)  // the ring's addresses are retired with it
    if (--*p.rings == 0) g_retired.push_back(p);
  delete r;
}

// a ring takes the pieces it maps (under g_pool_mu)
void hold_pieces(const std::vector<ffmp_piece>& v) {
  std::lock_guard<std::mutex> lk(g_pool_mu);
  for (const ffmp_piece& p : v) ++*p.rings;
}

// restores the caller's current device on scope exit
struct DeviceScope {
  int prev = -1;
  explicit DeviceScope(int d) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != d) (void)hipSetDevice(d);
  }
  ~DeviceScope() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

struct RingGeom {
  size_t gran, piece, stride;
  int per_slot;
  bool pairing;
  int scale;  // partner bytes per slot byte the raster writes in lockstep: 1 (float32 layout) or 2 (compact)
};

int ring_geom(int32_t device, int64_t slot_bytes, const void* partner, int64_t partner_bytes, RingGeom* g) {
  int vmm = 0;
  if (hipDeviceGetAttribute(&vmm, hipDeviceAttributeVirtualMemoryManagementSupported, device) != hipSuccess || !vmm)
    return fail(FFMP_E_HIP, "ffmp_ring: device %d has no virtual memory management", device);
  hipMemAllocationProp prop = dev_prop(device);
  hipError_t e = hipMemGetAllocationGranularity(&g->gran, &prop, hipMemAllocationGranularityMinimum);
  if (e != hipSuccess || g->gran == 0) return fail(FFMP_E_HIP, "hipMemGetAllocationGranularity: %s", hipGetErrorString(e));
  // pieces: 1 GiB for slots of >= 2 GiB (the pairing resolution), else one piece per slot
  const size_t slot_g = ((size_t)slot_bytes + g->gran - 1) / g->gran * g->gran;
  g->piece = slot_g >= (2ull << 30) ? (1ull << 30) : slot_g;
  g->per_slot = (int)((slot_g + g->piece - 1) / g->piece);
  g->stride = g->piece * (size_t)g->per_slot;
  g->pairing = partner != nullptr && g->piece >= (256ull << 20);
  // The raster writes cell q of a slot and of the partner (the potential plane) in lockstep: the
  // same byte offset in the float32 layout, twice the offset for compact uint8 frames beside a
  // binary16 plane — the ratio of the plane to one slot (rounded: a rebuild passes the stride).
  g->scale = partner && partner_bytes >= (int64_t)(1.5 * (double)slot_bytes) ? 2 : 1;
  return FFMP_OK;
}

void pool_put(const std::vector<ffmp_piece>& v) {
  std::lock_guard<std::mutex> lk(g_pool_mu);
  for (const ffmp_piece& p : v) g_pieces.push_back(p);
}

// a two-stream probe at or above this is a well-paired piece (MI355X: 6.7-7.0 TB/s paired
// well, 4.5-5.6 badly; tools/pair_alias_probe.hip)
constexpr double kPairFastGBs = 6200.0;
#ifndef FFMP_PAIR_ACCEPT
#define FFMP_PAIR_ACCEPT 0.93  // a piece is taken when its probe is within this factor of the best seen
#endif
constexpr double kPairAccept = FFMP_PAIR_ACCEPT;

// Pieces beyond the ones a ring needs (pairing candidates) only while the device keeps
// max(8 GiB, 5 %) free beside them.
bool room_for(size_t bytes) {
  size_t free_b = 0, total_b = 0;
  if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) return false;
  const size_t reserve = std::max((size_t)8 << 30, total_b / 20);
  return free_b > bytes + reserve;
}

// Fill r->pieces[pos] for every pos with need[pos] set: candidates from the pool first (at most
// 6 per position), then fresh pieces; with a partner, the first piece whose two-stream store
// probe against the partner bytes written beside it is within 7 % of the best probe seen
// (after >= 3 probes), else the best of 12.  Pieces held by a ring are never candidates.
// Retired pieces become reusable only after a device synchronize that follows their
// retirement: snapshot (and remove) this device's retired pieces under the lock, THEN
// synchronize, then pool exactly that snapshot.  A ring dropped by another thread after the
// snapshot (e.g. a DLPack deleter while ctypes has released the GIL) stays retired until the
// next call, so its in-flight writes can never land in a piece handed out (or released) after
// this.  The caller has made `device` current.
int drain_retired(int32_t device) {
  std::vector<ffmp_piece> retired;
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    for (size_t k = 0; k < g_retired.size();) {
      if (g_retired[k].device == device) {
        retired.push_back(g_retired[k]);
        g_retired.erase(g_retired.begin() + k);
      } else {
        ++k;
      }
    }
  }
  // every launch issued before the snapshot's rings died has finished once this returns
  if (hipDeviceSynchronize() != hipSuccess) {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    for (const ffmp_piece& p : retired) g_retired.push_back(p);
    return fail(FFMP_E_HIP, "ffmp_ring: hipDeviceSynchronize failed");
  }
  std::lock_guard<std::mutex> lk(g_pool_mu);
  for (const ffmp_piece& p : retired) g_pieces.push_back(p);
  return FFMP_OK;
}

int choose_pieces(ffmp_ring* r, const RingGeom& g, const std::vector<char>& need, const char* partner,
                  int64_t partner_bytes) {
  const int32_t device = r->device;
  std::vector<ffmp_piece> cand;
  if (const int rc = drain_retired(device)) return rc;
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    for (size_t k = 0; k < g_pieces.size();) {
      if (g_pieces[k].device == device && g_pieces[k].bytes == g.piece) {
        cand.push_back(g_pieces[k]);
        g_pieces.erase(g_pieces.begin() + k);
      } else {
        ++k;
      }
    }
  }
  hipStream_t s = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  struct Cleanup {
    hipStream_t& s; hipEvent_t& a; hipEvent_t& b;
    ~Cleanup() { if (a) (void)hipEventDestroy(a); if (b) (void)hipEventDestroy(b); if (s) (void)hipStreamDestroy(s); }
  } cleanup{s, e0, e1};
  if (g.pairing && (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess ||
                    hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess)) {
    pool_put(cand);
    return fail(FFMP_E_HIP, "ffmp_ring: stream/event creation failed");
  }
  // on failure: the candidates AND the pieces already chosen for earlier positions go back to the pool
  auto give_back = [&](size_t upto) {
    for (size_t q = 0; q < upto; ++q)
      if (need[q] && r->pieces[q].h) {
        cand.push_back(r->pieces[q]);
        r->pieces[q] = ffmp_piece{};
      }
    pool_put(cand);
  };
  int todo = 0;
  for (char n : need) todo += n != 0;
  // fresh pieces beyond need are the price of pairing (capped under an HBM budget).  Round 4: up to
  // one extra candidate per position (was one per two): with half, the search ran out of fresh
  // pieces on about half of fresh C3 processes (100 of 100 used) and the last slot's positions took
  // whatever was left — one slot 20 % slower, the metric -2.5 % (profiles/r04h_slot_repair.txt); the
  // unchosen pieces go back to the device afterwards (ffmp_ring_pool_trim), and only while
  // max(8 GiB, 5 %) of HBM stays free (room_for)
  const int32_t extra = ffmp_detail::g_ring_extra.load();
  const int max_new = todo + (extra > 0 ? extra - 1 : todo + 8);
  // best probe seen against this partner plane: the scale "fast" is judged against
  double ref = g.pairing ? pair_ref_get(device, g.scale, partner) : 0.0;
  bool found_fast = false;
  int fresh = 0;
  hipError_t e = hipSuccess;
  for (size_t pos = 0; pos < need.size(); ++pos) {
    if (!need[pos]) continue;
    const int j = (int)(pos % (size_t)g.per_slot);
    const size_t off = (size_t)j * g.piece * (size_t)g.scale;  // the partner bytes written beside piece j
    char* pb = g.pairing ? (char*)partner + off : nullptr;
    // slot bytes of piece j that have partner bytes beside them (the probe writes scale x these)
    const size_t pbytes = g.pairing && (int64_t)off < partner_bytes
                              ? std::min(g.piece, (size_t)(partner_bytes - (int64_t)off) / (size_t)g.scale) : 0;
    // no probe has found a fast pair in the first 12: the partner sits where nothing pairs
    // well (seen at C5), so stop paying for probes and extra pieces
    const bool test = g.pairing && pbytes >= (64u << 20) && (found_fast || r->pieces_tested < 12);
    int pick = -1, here = 0;
    double pick_gbs = -1.0;
    size_t k = 0;
    for (;;) {
      int c = -1;
      if (k < cand.size() && k < 6) {
        c = (int)k++;
      } else if (fresh < max_new && (fresh < todo || room_for(g.piece))) {
        ffmp_piece p;
        if ((e = new_piece(device, g.piece, g.gran, &p)) != hipSuccess) {
          (void)hipGetLastError();
          if (pick >= 0 || !cand.empty()) break;  // out of memory: settle for what there is
          give_back(pos);
          size_t free_b = 0, total_b = 0;
          (void)hipMemGetInfo(&free_b, &total_b);
          return fail(FFMP_E_HIP, "ffmp_ring: hipMemCreate/map of a %zu-byte piece: %s (device free %zu of %zu B)",
                      g.piece, hipGetErrorString(e), free_b, total_b);
        }
        ++fresh;
        cand.push_back(p);
        c = (int)cand.size() - 1;
        k = cand.size();
      } else {
        break;
      }
      if (!test) {
        pick = c;
        break;
      }
      const double gbs = pair_gbs(cand[c].home, pb, pbytes, g.scale, s, e0, e1);
      if (gbs < 0.0) {
        give_back(pos);
        return fail(FFMP_E_HIP, "ffmp_ring: pairing probe failed: %s", hipGetErrorString(hipGetLastError()));
      }
      ++r->pieces_tested;
      ++here;
      if (gbs >= kPairFastGBs) found_fast = true;
      if (gbs > ref) {
        ref = gbs;
        pair_ref_put(device, g.scale, partner, gbs);
      }
      if (gbs > pick_gbs) {
        pick = c;
        pick_gbs = gbs;
      }
      // accept within 7 % of the best probe seen against this partner plane (this ring or an earlier
      // one / a rebuild), and
      // never below kPairFastGBs: slot 0's positions come first, and judged only against the
      // handful of probes seen so far they took badly paired pieces (round 2: slot 0 ~10 % slower
      // than every other slot on three boxes, and again after a rebuild)
      if ((r->pieces_tested >= 3 || ref > kPairFastGBs) && pick_gbs >= std::max(kPairAccept * ref, kPairFastGBs)) break;
      if (here >= 12) break;  // bounded search: keep the best seen
    }
    if (pick < 0) {
      give_back(pos);
      return fail(FFMP_E_HIP, "ffmp_ring: no piece available");
    }
    if (test) {
      r->pair_gbs_min = r->pair_gbs_min > 0 ? std::min(r->pair_gbs_min, pick_gbs) : pick_gbs;
      r->pair_gbs_max = std::max(r->pair_gbs_max, pick_gbs);
    }
    r->pieces[pos] = cand[pick];
    cand.erase(cand.begin() + pick);
  }
  r->pieces_new += fresh;
  pool_put(cand);
  return FFMP_OK;
}

// reserve the ring's own addresses and map slots 0..W-1, then slot 0's pieces again
int ring_map(ffmp_ring* r, const RingGeom& g) {
  // aligned to the piece (up to 1 GiB) so that every piece maps with the largest page fragments
  hipError_t e = hipMemAddressReserve((void**)&r->va, r->vbytes, va_align(g.piece, g.gran), nullptr, 0);
  if (e != hipSuccess) return fail(FFMP_E_HIP, "ffmp_ring: hipMemAddressReserve: %s", hipGetErrorString(e));
  ffmp_detail::note_va(r->device, r->vbytes);
  for (int v = 0; v <= r->slots; ++v) {
    const int slot = v % r->slots;
    for (int j = 0; j < g.per_slot; ++j) {
      const ffmp_piece& p = r->pieces[(size_t)slot * g.per_slot + j];
      char* at = r->va + (size_t)v * r->stride + (size_t)j * g.piece;
      e = hipMemMap(at, g.piece, 0, p.h, 0);
      if (e == hipSuccess) {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        p.maps->push_back(at);  // unmapped only when the piece's memory is released (pool trim)
      }
      if (e == hipSuccess) {
        hipMemAccessDesc acc = {};
        acc.location = dev_prop(r->device).location;
        acc.flags = hipMemAccessFlagsProtReadWrite;
        e = hipMemSetAccess(at, g.piece, &acc, 1);
      }
      if (e != hipSuccess) return fail(FFMP_E_HIP, "ffmp_ring: hipMemMap: %s", hipGetErrorString(e));  // never reused
    }
  }
  return FFMP_OK;
}

}  // namespace

extern "C" {

int ffmp_ring_create(int32_t device, int64_t slot_bytes, int32_t slots, const void* partner, int64_t partner_bytes,
                     ffmp_ring_t** ring, void** base, int64_t* slot_stride) {
  if (!ring || !base || !slot_stride) return fail(FFMP_E_ARG, "ffmp_ring_create: NULL output pointer");
  *ring = nullptr;
  *base = nullptr;
  if (slot_bytes <= 0 || slots < 2) return fail(FFMP_E_ARG, "ffmp_ring_create: slot_bytes > 0 and slots >= 2 required");
  if (partner && partner_bytes <= 0) return fail(FFMP_E_ARG, "ffmp_ring_create: partner_bytes must be > 0");
  DeviceScope scope(device);
  RingGeom g;
  if (const int rc = ring_geom(device, slot_bytes, partner, partner_bytes, &g)) return rc;
  std::unique_ptr<ffmp_ring> r(new ffmp_ring());
  r->device = device;
  r->slots = slots;
  r->scale = g.scale;
  r->stride = g.stride;
  r->vbytes = g.stride * (size_t)(slots + 1);
  r->pieces.resize((size_t)slots * g.per_slot);
  const std::vector<char> need(r->pieces.size(), 1);
  if (const int rc = choose_pieces(r.get(), g, need, (const char*)partner, partner_bytes)) return rc;
  if (const int rc = ring_map(r.get(), g)) {
    pool_put(r->pieces);
    return rc;
  }
  hold_pieces(r->pieces);
  r->refs = 1;
  *base = r->va;
  *slot_stride = (int64_t)r->stride;
  *ring = r.release();
  return FFMP_OK;
}

int ffmp_ring_rebuild(ffmp_ring_t* old, uint64_t replace_mask, const void* partner, int64_t partner_bytes,
                      ffmp_ring_t** ring, void** base, int64_t* slot_stride) {
  if (!old || !ring || !base || !slot_stride) return fail(FFMP_E_ARG, "ffmp_ring_rebuild: NULL argument");
  *ring = nullptr;
  *base = nullptr;
  if (old->slots > 64) return fail(FFMP_E_ARG, "ffmp_ring_rebuild: more than 64 slots");
  if (partner && partner_bytes <= 0) return fail(FFMP_E_ARG, "ffmp_ring_rebuild: partner_bytes must be > 0");
  DeviceScope scope(old->device);
  RingGeom g;
  if (const int rc = ring_geom(old->device, (int64_t)old->stride, partner, partner_bytes, &g)) return rc;
  if (g.stride != old->stride) return fail(FFMP_E_ARG, "ffmp_ring_rebuild: geometry changed");
  // the partner ratio is the ring's, fixed at create: guessing it again from old->stride (slots
  // rounded up to whole pieces) could flip it, e.g. for compact slots of 2-2.25 GiB
  if (partner) g.scale = old->scale;
  std::unique_ptr<ffmp_ring> r(new ffmp_ring());
  r->device = old->device;
  r->slots = old->slots;
  r->scale = old->scale;
  r->stride = old->stride;
  r->vbytes = old->vbytes;
  r->pieces.resize(old->pieces.size());
  std::vector<char> need(r->pieces.size(), 0);
  for (size_t pos = 0; pos < old->pieces.size(); ++pos) {
    const int slot = (int)(pos / (size_t)g.per_slot);
    if ((replace_mask >> slot) & 1u)
      need[pos] = 1;  // old's piece stays held by old, so it is not a candidate
    else
      r->pieces[pos] = old->pieces[pos];
  }
  if (const int rc = choose_pieces(r.get(), g, need, (const char*)partner, partner_bytes)) return rc;
  if (const int rc = ring_map(r.get(), g)) {
    // the kept pieces still belong to `old`; give back only the new ones
    std::vector<ffmp_piece> fresh;
    for (size_t pos = 0; pos < need.size(); ++pos)
      if (need[pos]) fresh.push_back(r->pieces[pos]);
    pool_put(fresh);
    return rc;
  }
  // `old` stays whole and usable; the kept pieces are now held by both rings
  hold_pieces(r->pieces);
  r->pieces_new += old->pieces_new;
  r->pieces_tested += old->pieces_tested;
  r->refs = 1;
  *base = r->va;
  *slot_stride = (int64_t)r->stride;
  *ring = r.release();
  return FFMP_OK;
}

int ffmp_ring_destroy(ffmp_ring_t* ring) {
  if (ring) ring_unref(ring);
  return FFMP_OK;
}

int ffmp_ring_info(const ffmp_ring_t* ring, double* out, int32_t cap) {
  if (!ring || !out || cap < 5) return fail(FFMP_E_ARG, "ffmp_ring_info: ring/out NULL or cap < 5");
  out[0] = (double)ring->pieces.size();
  out[1] = (double)ring->pieces_new;
  out[2] = (double)ring->pieces_tested;
  out[3] = ring->pair_gbs_min;
  out[4] = ring->pair_gbs_max;
  if (cap < 6) return 5;
  out[5] = (double)ring->scale;
  return 6;
}

int64_t ffmp_ring_va_reserved(int32_t device) {
  if (device < 0 || device >= ffmp_detail::kVaDevices) return fail(FFMP_E_ARG, "ffmp_ring_va_reserved: device out of range");
  return ffmp_detail::g_va_reserved[device].load();
}

int64_t ffmp_ring_pool_bytes(int32_t device) {
  std::lock_guard<std::mutex> lk(g_pool_mu);
  int64_t b = 0;
  for (const std::vector<ffmp_piece>* v : {&g_pieces, &g_retired})
    for (const ffmp_piece& p : *v)
      if (p.device == device || device < 0) b += (int64_t)p.bytes;
  return b;
}

int ffmp_ring_pair_forget(int32_t device, const void* partner) {
  if (device < 0) return fail(FFMP_E_ARG, "ffmp_ring_pair_forget: device must be >= 0");
  std::lock_guard<std::mutex> lk(g_pool_mu);
  const size_t before = g_pair_ref.size();
  g_pair_ref.erase(std::remove_if(g_pair_ref.begin(), g_pair_ref.end(),
                                  [device, partner](const PairRef& p) {
                                    return p.device == device && (!partner || p.partner == partner);
                                  }),
                   g_pair_ref.end());
  return (int)(before - g_pair_ref.size());
}

int ffmp_ring_pair_refs(int32_t device) {
  std::lock_guard<std::mutex> lk(g_pool_mu);
  int n = 0;
  for (const PairRef& p : g_pair_ref) n += p.device == device;
  return n;
}

int ffmp_ring_pool_trim(int32_t device, int64_t keep_bytes, int64_t* released) {
  if (released) *released = 0;
  if (device < 0) return fail(FFMP_E_ARG, "ffmp_ring_pool_trim: device must be >= 0");
  DeviceScope scope(device);
  // pieces of rings dropped while kernels may still write them become pool pieces only after a
  // device synchronize; their memory is released after that too
  if (const int rc = drain_retired(device)) return rc;
  std::vector<ffmp_piece> victims;
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    // (the pairing references stay: live instances' rebuilds keep judging on their own scale; an
    // owner forgets its partner plane's references when it frees the plane, ffmp_ring_pair_forget)
    int64_t kept = 0;
    for (size_t k = 0; k < g_pieces.size();) {
      ffmp_piece& p = g_pieces[k];
      if (p.device != device || kept + (int64_t)p.bytes <= std::max<int64_t>(keep_bytes, 0)) {
        if (p.device == device) kept += (int64_t)p.bytes;
        ++k;
        continue;
      }
      victims.push_back(p);
      g_pieces.erase(g_pieces.begin() + k);
    }
  }
  int rc = FFMP_OK;
  int64_t freed = 0;
  for (ffmp_piece& p : victims) {
    // every mapping (home + the dead rings' slots) goes; the reservations stay, never reused
    bool ok = true;
    for (char* at : *p.maps)
      if (hipMemUnmap(at, p.bytes) != hipSuccess) ok = false;
    if (ok && hipMemRelease(p.h) == hipSuccess) {
      freed += (int64_t)p.bytes;
      delete p.maps;
      delete p.rings;
    } else {
      (void)hipGetLastError();
      rc = fail(FFMP_E_HIP, "ffmp_ring_pool_trim: unmapping / releasing a %zu-byte piece failed", p.bytes);
    }
  }
  if (released) *released = freed;
  return rc;
}

static void dl_delete(DLManagedTensor_* mt) {
  DLHolder_* h = (DLHolder_*)mt->manager_ctx;
  if (h->owner) ring_unref(h->owner);
  free(h);
}

void* ffmp_dlpack(void* data, int32_t device_type, int32_t device_id, int32_t ndim, const int64_t* shape,
                  const int64_t* strides, int32_t bits, ffmp_ring_t* owner) {
  if (!data || ndim < 1 || ndim > 8 || !shape || !strides || (bits != 8 && bits != 16 && bits != 32 && bits != 64)) {
    fail(FFMP_E_ARG, "ffmp_dlpack: bad arguments");
    return nullptr;
  }
  DLHolder_* h = (DLHolder_*)calloc(1, sizeof(DLHolder_));
  if (!h) {
    fail(FFMP_E_ARG, "ffmp_dlpack: out of host memory");
    return nullptr;
  }
  for (int d = 0; d < ndim; ++d) {
    h->dims[d] = shape[d];
    h->dims[8 + d] = strides[d];
  }
  h->mt.dl_tensor.data = data;
  h->mt.dl_tensor.device = {device_type, device_id};
  h->mt.dl_tensor.ndim = ndim;
  // 8-bit elements are uint8 (the compact frames, FFMP_OBS_U8F16); wider ones are floats
  h->mt.dl_tensor.dtype = {(uint8_t)(bits == 8 ? 1 /* kDLUInt */ : 2 /* kDLFloat */), (uint8_t)bits, 1};
  h->mt.dl_tensor.shape = h->dims;
  h->mt.dl_tensor.strides = h->dims + 8;
  h->mt.manager_ctx = h;
  h->mt.deleter = dl_delete;
  h->owner = owner;
  if (owner) __atomic_add_fetch(&owner->refs, 1, __ATOMIC_ACQ_REL);
  return &h->mt;
}

}  // extern "C"
