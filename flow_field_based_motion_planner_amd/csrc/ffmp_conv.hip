// ffmp_conv.hip — the learner's dominant convolution as a hand-written CDNA4 MFMA kernel.
//
// The reference Network (/root/reference/src/train.py:231-303) spends ~80 % of its FLOPs in
// conv2 (32 -> 64 channels, 32 x 32 kernel, 69^2 -> 38^2, stride 1, no padding: 6.06 GFLOP per
// sample forward).  This is that convolution as an implicit GEMM on v_mfma_f32_32x32x16_bf16
// (bf16 operands, fp32 accumulation), with the bias and ReLU fused into the epilogue:
//
//   y[b, p, n] = relu(bias[n] + sum_{ky, kx, c} x[b, yp + ky, xp + kx, c] * w[ky, kx, n, c])
//
// GEMM view: M = output positions p = (yp, xp) of one sample, N = output channels, K = taps x
// input channels.  Layouts (all contiguous): x NHWC bf16 [B][H][W][C]; w bf16 [KH][KW][N][C]
// (a tap's N x C block is the B operand: lane (r, h) reads w[tap][nb*32 + r][s*16 + 8h .. +8],
// 16 contiguous bytes); y NHWC [B][Ho][Wo][N], fp32 or bf16.
//
// Tiling.  A workgroup (4 waves) owns PT = 4 * MBW * 32 consecutive output positions of one
// sample and all N channels; a wave owns MBW 32-position blocks x NB 32-channel blocks (acc:
// MBW * NB * 16 fp32 per lane).  For a fixed kernel row ky the positions read input rows
// yp + ky only, so the A operand comes from a ring of input rows in LDS: the rows
// [y_first + ky, y_last + ky] of the tile, one new row per ky (loaded into registers during ky,
// written after it), i.e. every input byte crosses L2 -> LDS once per workgroup.  The A
// fragment of lane (r, h) at tap (ky, kx), k-step s is 16 contiguous bytes of the ring:
// row (yp + ky) % RING, column xp + kx, channels s*16 + 8h .. +8 — the per-lane row/column base
// plus a wave-uniform tap offset.  B fragments (a tap is N * C * 2 = 4 KB, shared by every
// workgroup) come from global memory through L1/L2 into registers, one tap ahead.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <utility>

#include "ffmp.h"

namespace ffmp_detail {
int fail(int code, const char* fmt, ...);  // ffmp_kernels.hip (sets ffmp_last_error())
// ffmp_conv2d_check: run every shape check of a launch, then return before launching
thread_local bool t_conv_dry = false;
// the MFMA shape of the convolution kernels that have both (FFMP_TUNE_CONV_MFMA): 0 = each kernel's
// default (32x32x16 for the forwards, the data gradient and conv2's weight gradient: profiles/r06a_conv_ab.txt,
// r06b_conv_ab.txt — the 16x16x32 stream ran 6-50 % slower there, the samples-as-M data gradient within
// the run-to-run spread; 16x16x32 for the other weight gradients, 6-15 % faster, and the small-image
// kernel's padded data gradients, 3-6 %: profiles/r06j_conv_ab_*_ms16.txt), 16 = 16x16x32, 32 = 32x32x16
int g_conv_mfma = 0;
int mfma_for(int dflt) { return g_conv_mfma ? g_conv_mfma : dflt; }
int conv_mfma_swap(int v) {
  const int prev = g_conv_mfma;
  g_conv_mfma = v;
  return prev;
}
// the row-ring forward's B operand through LDS (FFMP_TUNE_CONV_LB): 0 = off (default), 1 = on where it fits
// (conv2's forward 1.35 against 1.28 ms: the per-tap barrier costs more than the shared weight loads
// save, profiles/r06b_conv_ab.txt)
int g_conv_lb = 0;
int conv_lb_swap(int v) {
  const int prev = g_conv_lb;
  g_conv_lb = v;
  return prev;
}
// the weight gradient's operand reads one k-step ahead (FFMP_TUNE_CONV_WGPF): 0 = by FFMP_WGRAD_PREFETCH, 1 = on
int g_conv_wgpf = 0;
int conv_wgpf_swap(int v) {
  const int prev = g_conv_wgpf;
  g_conv_wgpf = v;
  return prev;
}
// conv2-shaped forwards with pinned load schedules (FFMP_TUNE_CONV_BA2): 0 = default (off), 1 = B
// fragments two taps ahead, 2 = one tap ahead
int g_conv_ba2 = 0;
int conv_ba2_swap(int v) {
  const int prev = g_conv_ba2;
  g_conv_ba2 = v;
  return prev;
}
// the row-ring forward's default launch with pinned load schedules (FFMP_TUNE_CONV_PIN): 0 = off, 1 = on
int g_conv_pin = 0;
int conv_pin_swap(int v) {
  const int prev = g_conv_pin;
  g_conv_pin = v;
  return prev;
}
// the weight gradient's LDS-DMA double-buffered stages (FFMP_TUNE_CONV_WGDMA): 0 = by shape (with the k-step
// prefetch where the kernel runs one workgroup per CU), 1 = on, 2 = on with the prefetch, 3 = off, 4 = the
// 32 -> 64 layer with 4 taps per wave (two workgroups per CU) on prefetched LDS-DMA stages
int g_conv_wgdma = 0;
int conv_wgdma_swap(int v) {
  const int prev = g_conv_wgdma;
  g_conv_wgdma = v;
  return prev;
}
// planar ring slots for the row-ring forward (FFMP_TUNE_CONV_PLANAR): 0 = off (default), 1 = on
int g_conv_planar = 0;
int conv_planar_swap(int v) {
  const int prev = g_conv_planar;
  g_conv_planar = v;
  return prev;
}
// 32-position blocks per wave of the row-ring forward (FFMP_TUNE_CONV_MBW): 0 = by the grid-fill
// model (pick_mbw), 1 / 2 / 3 / 4 forced
int g_conv_mbw = 0;
int conv_mbw_swap(int v) {
  const int prev = g_conv_mbw;
  g_conv_mbw = v;
  return prev;
}
// kernel rows per ring step of the row-ring forward (FFMP_TUNE_CONV_KYS): 0 = default (1), 1, 2 or 4
int g_conv_kys = 0;
int conv_kys_swap(int v) {
  const int prev = g_conv_kys;
  g_conv_kys = v;
  return prev;
}
}
using ffmp_detail::fail;
using ffmp_detail::t_conv_dry;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kWaves = 4;

// One input row's 16-byte chunks into registers.  cellb = bytes between two cells of the row in
// global memory: C * 2 (a plain NHWC row), or, for an input folded on the fly (FFMP_CONV_X_FOLD),
// the unfolded cell's (C / F) * 2 — folded cell x is then the C * 2 bytes starting at unfolded cell
// x (dword-aligned, read as dwords).
template <int C, int NR = 4>
__device__ __forceinline__ void load_row_regs(const char* __restrict__ src, int chunks, int cellb, uint4 (&buf)[NR]) {
  constexpr int CPC = C / 8;  // 16-byte chunks per cell
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int q = threadIdx.x + 256 * i;
    if (q >= chunks) continue;
    if (!src) {
      buf[i] = uint4{0u, 0u, 0u, 0u};
    } else if (cellb == C * 2) {
      buf[i] = *(const uint4*)(src + 16 * (size_t)q);
    } else {
      const uint32_t* p = (const uint32_t*)(src + (size_t)(q / CPC) * cellb + 16 * (q % CPC));
      buf[i] = uint4{p[0], p[1], p[2], p[3]};
    }
  }
}

// global geometry of the input rows: cell bytes and row bytes (see load_row_regs)
template <int C>
__device__ __forceinline__ int2 in_geom(int W, int dx, int flags) {
  if (flags & FFMP_CONV_X_FOLD) return int2{(C / dx) * 2, (W + dx - 1) * (C / dx) * 2};
  return int2{C * 2, W * C * 2};
}

// LDS images of NHWC rows are padded by 16 bytes after every 256: column col starts at
// cell_off(col) = col * C * 2 + (col / (256 / (C * 2))) * 16.  The A fragment of lane r reads one
// 16-byte chunk of column xcol + r; unpadded, the columns of a ds_read_b128 lane group (C * 2 bytes
// apart) fall on 2 (C = 64) or 4 (C = 32) of the 16 bank quads — 8- / 4-way conflicts; padded, the
// 16 lanes {0-3, 12-15, 20-27} of a group take 16 distinct quads, and the chunk offsets stay
// compile-time constants (no per-read address arithmetic, unlike an XOR swizzle).
template <int C>
__host__ __device__ __forceinline__ int cell_off(int col) {
  constexpr unsigned CPR = 256 / (C * 2);  // columns per 256 bytes
  // unsigned: col >= 0 at every call, and a signed division by 4 costs the kernels' inner loops three
  // VALU per operand address (ashr / lshr / add before the shift)
  return (int)((unsigned)col * (C * 2) + ((unsigned)col / CPR) * 16);
}
template <int C>
__host__ __device__ __forceinline__ int lds_pitch(int W) {  // bytes of one padded row image
  return cell_off<C>(W - 1) + C * 2;
}

template <int C, int NR = 4>
__device__ __forceinline__ void store_row_lds(char* dst, int chunks, const uint4 (&buf)[NR]) {
  constexpr int CPC = C / 8;  // 16-byte chunks per column
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int q = threadIdx.x + 256 * i;
    if (q < chunks) *(uint4*)(dst + cell_off<C>(q / CPC) + 16 * (q % CPC)) = buf[i];
  }
}

// Planar ring slots (FFMP_TUNE_CONV_PLANAR, 32x32x16 forwards): a slot holds the row's 16-byte chunk j
// of every cell contiguously in plane j (cell col at j * plane + 16 col), plane = (W + PAD) * 16 bytes
// (PAD: a zero cell at column W of every plane).  Lane r of an A fragment reads chunk j of column
// x0 + r: 16 consecutive columns are 16 consecutive quads, so every ds_read_b128 lane group
// ({0-3, 12-15, 20-27}, {4-11, 16-19, 28-31}: MI355X_MICROARCH.md LDS table) is conflict-free for ANY
// first column x0 — the padded cell layout above is conflict-free only for x0 = 0 mod 4, and its
// conflicts cost conv2's forward 46 % of its LDS cycles (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE,
// profiles/r06f_conv_pmc.txt; tools/lds_bank_model.py: 7.6 LDS cycles per read against 4).  A
// 32-position block that wraps from output row y to y + 1 continues in the next slot: the slot
// pitch is padded to = 16 Wo (mod 256), so the wrapped lanes land on the quads the row would have
// continued on.
__host__ __device__ __forceinline__ int planar_plane(int W, bool pad) { return (W + (pad ? 1 : 0)) * 16; }
template <int C>
__host__ __device__ __forceinline__ int planar_pitch(int W, int Wo, bool pad) {
  const int base = (C / 8) * planar_plane(W, pad);
  return base + (((Wo * 16 - base) % 256) + 256) % 256;
}
template <int C, int NR = 4>
__device__ __forceinline__ void store_row_planar(char* dst, int chunks, int plane, const uint4 (&buf)[NR]) {
  constexpr int CPC = C / 8;
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int q = threadIdx.x + 256 * i;
    if (q < chunks) *(uint4*)(dst + (q % CPC) * plane + 16 * (q / CPC)) = buf[i];
  }
}

// The B fragment of lane (r, h) for tap t, channel block nb, k-step s: 8 bf16 of weight row
// n = nb * 32 + r, channels s * 16 + 8h .. +8.  WF = false: w [KH][KW][N][C] (the fragment's 64
// lanes touch 32 rows 2 * C bytes apart, i.e. 32 cache lines for 1 KiB); WF = true
// (FFMP_CONV_W_FRAG): w in fragment order [KH][KW][N / 32][C / 16][2][32][8], the 64 lanes read
// 1 KiB contiguous — conv_small_kernel 0.48 -> 0.40 ms over the Network's conv3 / conv4 shapes at
// B = 256, conv2's forward unchanged (profiles/r05sm_conv_small.txt, r05k_conv_fwd_probes.txt)
template <int C, int NB, bool WF>
__device__ __forceinline__ bf16x8 load_bfrag(const __bf16* __restrict__ w, int t, int nb, int s, int r, int h) {
  if constexpr (WF)
    return *(const bf16x8*)(w + (size_t)(((t * NB + nb) * (C / 16) + s) * 2 + h) * 256 + r * 8);
  else
    return *(const bf16x8*)(w + ((size_t)(t * NB * 32 + nb * 32 + r) * C + s * 16 + h * 8));
}

// Implicit zero padding of `pad` cells on every side: logical input rows/columns [pad, pad + H/W)
// hold the tensor, the rest are zero.  A ring slot holds the W real cells of a row (zeros for a row
// outside the tensor); with PAD, a lane whose logical column falls outside [pad, pad + W) reads a
// clamped address and zeroes the fragment (a select instead of 2 pad columns of LDS per slot:
// the data gradient's slots shrink from 100 to 38 cells, so 512-position tiles fit twice per CU).
// The ky loop runs only over kernel rows for which some row of the tile touches the tensor, and a
// wave skips the MFMAs of kernel rows its own positions never see (the data gradient's k - 1 zero
// border: ~12 % of its work).  Kernel column kx reads input column xp + kx * dx (dx > 1: the
// x-dilated form a 1- or 2-channel convolution takes after its kernel columns are folded into
// channels, conv_mfma.fold_input).
// B fragments: 1 = the next tap's loaded into a copy that replaces the current set (the copy made
// every tap wait for them after one k-step of MFMAs: vmcnt(0) at the top of each tap), 2 = two sets
// that swap roles (the kx loop unrolled by two), each waited for a whole tap after its request.
// 0 (default): 2 for one channel block (NB = 1: the data gradient 3.20 -> 3.10-3.15 ms, the folded
// conv1 0.414 -> 0.393 ms at B = 256), 1 for two (NB = 2: conv2's forward has 233 of its 256
// registers in use and ran 1.37 -> 1.67 ms with the second set; profiles/r04q_conv_prefetch.txt).
#ifndef FFMP_CONV_BAHEAD
#define FFMP_CONV_BAHEAD 0
#endif

#ifndef FFMP_CONV_FWD_OCC
#define FFMP_CONV_FWD_OCC 2  // workgroups per CU the forward kernel is compiled for
#endif
// MFMA shape MS: 32 = v_mfma_f32_32x32x16_bf16 (32-position x 32-channel blocks, k-steps of 16
// channels), 16 = v_mfma_f32_16x16x32_bf16 (16 x 16 blocks, k-steps of 32) at the same output tile
// per wave — the same FLOPs, A/B bytes and accumulator registers, but the chip holds a higher clock
// on the 16x16x32 stream (MI355X_MICROARCH.md, DVFS give-back item 7: ~1.12-1.15x the FLOP/s on
// random data).  Lane l of a 16x16x32 operand holds row l & 15, k = 8 (l >> 4) .. +8; its C/D
// element i is row 4 (l >> 4) + i, column l & 15.
template <int MS>
struct Mfma;
template <>
struct Mfma<32> {
  typedef f32x16 acc_t;
  static constexpr int KS = 16, NACC = 16;
  static __device__ __forceinline__ acc_t mma(bf16x8 a, bf16x8 b, acc_t c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ int row(int i, int kh) { return (i & 3) + 8 * (i >> 2) + 4 * kh; }
};
template <>
struct Mfma<16> {
  typedef f32x4 acc_t;
  static constexpr int KS = 32, NACC = 4;
  static __device__ __forceinline__ acc_t mma(bf16x8 a, bf16x8 b, acc_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ int row(int i, int kh) { return 4 * kh + i; }
};


// B fragment (output-channel block nb of MS, k-step s of Mfma<MS>::KS channels) of lane (r, kh) at tap
// t.  MS = 16 reads w[t][n = nb * 16 + r][s * 32 + 8 kh .. +8]: plain [KH][KW][N][C] at C = 32 is 16
// rows x 64 bytes = 1 KiB contiguous; in fragment order (WF, laid out for the 32x32x16 operand) the
// same 8 channels sit at ((t NB + nb / 2) (C / 16) + 2 s) 512 + 256 kh + ((nb & 1) 16 + r) 8: four
// 256-byte runs
template <int C, int NB, bool WF, int MS>
__device__ __forceinline__ bf16x8 load_bfrag_ms(const __bf16* __restrict__ w, int t, int nb, int s, int r, int kh) {
  if constexpr (MS == 32) {
    return load_bfrag<C, NB, WF>(w, t, nb, s, r, kh);
  } else if constexpr (WF) {
    return *(const bf16x8*)(w + (size_t)((t * NB + (nb >> 1)) * (C / 16) + 2 * s) * 512 + kh * 256 +
                            ((nb & 1) * 16 + r) * 8);
  } else {
    return *(const bf16x8*)(w + ((size_t)(t * NB * 32 + nb * 16 + r) * C + s * 32 + kh * 8));
  }
}

// NRC: 16-byte row chunks per thread the next-row registers hold (ceil(row bytes / 4 KiB); 4 covers
// every shape, conv2's 4.4 KiB rows need 2: 8 registers fewer); BA: B fragments 1 or 2 taps ahead
// (0: 2 for one channel block, 1 for two — the 1-ahead set of conv2's forward waits on every tap's
// loads, the 2-ahead one needs the registers NRC = 2 frees); PIN: each tap's loads pinned ahead of
// its MFMAs by scheduling barriers (the scheduler otherwise sinks the next tap's B loads below half
// of the tap's MFMAs and waits on each A read one MFMA after issuing it: profiles/r06e_conv2_isa.txt)
template <int C, int NB, int MBW, bool PAD, bool WF, int MS = 32, int KYS = 1, int NRC = 4, int BA = 0, bool PIN = false,
          bool PL = false>
__global__ __launch_bounds__(256, FFMP_CONV_FWD_OCC) void conv_fwd_kernel(const __bf16* __restrict__ x, const __bf16* __restrict__ w,
                                                          const float* __restrict__ bias, void* __restrict__ y, int H,
                                                          int W, int KH, int KW, int pad, int dx, int RING, int flags) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  using M = Mfma<MS>;
  constexpr int N = NB * 32;
  constexpr int PT = kWaves * MBW * 32;
  constexpr int AM = MBW * 32 / MS, AN = N / MS;  // MFMA blocks per wave: positions x channels
  constexpr int KSTEPS = C / M::KS;                // k-steps per tap
  const int Ho = H + 2 * pad - KH + 1, Wo = W + 2 * pad - (KW - 1) * dx;
  const int b = blockIdx.y;
  const int P = Ho * Wo;
  const int p0 = blockIdx.x * PT;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & (MS - 1), kh = lane / MS;  // operand row, k-chunk of 8 channels
  const int rowbytes = W * C * 2;      // one tensor row (of the folded image with FFMP_CONV_X_FOLD)
  static_assert(!PL || MS == 32, "planar slots: 32x32x16 lane groups only");
  // its padded image (or its planes, PL) = one ring slot
  const int pitch = PL ? planar_pitch<C>(W, Wo, PAD) : lds_pitch<C>(W);
  const int plane = planar_plane(W, PAD);
  const int chunks = rowbytes / 16;    // <= 4 * 256 (host check)
  const int2 gin = in_geom<C>(W, dx, flags);  // the row's cell / row bytes in global memory
  const int zero_off = RING * pitch;   // a zero column (PAD: reads outside the tensor's columns)
  auto store_row = [&](char* dst, const auto& buf) {
    if constexpr (PL) store_row_planar<C>(dst, chunks, plane, buf);
    else store_row_lds<C>(dst, chunks, buf);
  };
  const int yf = p0 / Wo;
  const int yl = min(P - 1, p0 + PT - 1) / Wo;
  const char* xb = (const char*)x + (size_t)b * H * gin.y;
  // kernel rows whose input rows [yf + ky, yl + ky] meet the tensor rows [pad, pad + H) ...
  const int ky_lo = max(0, pad - yl), ky_hi = min(KH - 1, pad + H - 1 - yf);
  // ... and this wave's share of them (its positions' rows)
  const int pw0 = p0 + wave * MBW * 32;
  const int wyf = min(pw0, P - 1) / Wo, wyl = min(P - 1, pw0 + MBW * 32 - 1) / Wo;
  const int wk_lo = pw0 < P ? max(ky_lo, pad - wyl) : KH, wk_hi = min(ky_hi, pad + H - 1 - wyf);

  // this lane's output positions (clamped into the image; out-of-range ones are not stored):
  // output row, and input column of kernel column 0 relative to the tensor (xp - pad)
  int ypos[AM], xcol[AM];
#pragma unroll
  for (int mb = 0; mb < AM; ++mb) {
    const int m = min(pw0 + mb * MS + r, P - 1);
    ypos[mb] = m / Wo;
    xcol[mb] = m - ypos[mb] * Wo - pad;
  }
  auto row_src = [&](int yr) -> const char* {  // logical row -> tensor row, or nullptr (zeros)
    const int real = yr - pad;
    return (real >= 0 && real < H) ? xb + (size_t)real * gin.y : nullptr;
  };
  // ring rows for the first chunk of kernel rows
  for (int row = yf + ky_lo; row <= yl + min(ky_lo + KYS - 1, ky_hi); ++row) {
    uint4 buf[4];
    load_row_regs<C>(row_src(row), chunks, gin.x, buf);
    store_row(lds + (row % RING) * pitch, buf);
  }
  if constexpr (PL && PAD) {  // the zero cell of every plane of every slot
    for (int q = threadIdx.x; q < RING * (C / 8); q += 256)
      *(uint4*)(lds + (q / (C / 8)) * pitch + (q % (C / 8)) * plane + 16 * W) = uint4{0u, 0u, 0u, 0u};
  } else if (PAD && threadIdx.x < C / 8) {
    *(uint4*)(lds + zero_off + 16 * threadIdx.x) = uint4{0u, 0u, 0u, 0u};
  }
  __syncthreads();

  typename M::acc_t acc[AM][AN];
#pragma unroll
  for (int mb = 0; mb < AM; ++mb)
#pragma unroll
    for (int nb = 0; nb < AN; ++nb) acc[mb][nb] = typename M::acc_t{};

  // B fragments of the wave's first tap (wk_lo, 0); from then on loaded one tap ahead (the active
  // kernel rows [wk_lo, wk_hi] are consecutive, so the tap after t is t + 1, up to the wave's last
  // tap, which later loads re-read)
  const int t_last = min(wk_hi, KH - 1) * KW + KW - 1;
  auto load_b = [&](int t, bf16x8 (&dst)[AN][KSTEPS]) {
    t = min(t, t_last);
#pragma unroll
    for (int nb = 0; nb < AN; ++nb)
#pragma unroll
      for (int s = 0; s < KSTEPS; ++s) {
        dst[nb][s] = load_bfrag_ms<C, NB, WF, MS>(w, t, nb, s, r, kh);
      }
  };
  constexpr int kBAhead = BA > 0 ? BA : FFMP_CONV_BAHEAD > 0 ? FFMP_CONV_BAHEAD : (NB == 1 ? 2 : 1);
  bf16x8 bcur[AN][KSTEPS];
  bf16x8 bnx[AN][KSTEPS];  // kBAhead 2: the ping-pong partner of bcur
  load_b(min(wk_lo, KH - 1) * KW, bcur);

  // kernel rows in chunks of KYS per ring step: the chunk's rows are in the ring, the next chunk's
  // KYS rows are loaded into registers during it and written after it (KYS = 1: before the chunk's
  // barrier, into the ring's spare slot; KYS > 1: between two barriers, over the rows the chunk was
  // the last to read — ring = span + KYS - 1 slots, one barrier pair per KYS kernel rows)
  for (int ky0 = ky_lo; ky0 <= ky_hi; ky0 += KYS) {
    const int kyn = min(KYS, ky_hi - ky0 + 1);
    const int nnext = min(KYS, ky_hi - (ky0 + kyn) + 1);  // rows of the next chunk (<= 0: none)
    uint4 nrow[KYS][NRC];
#pragma unroll
    for (int j = 0; j < KYS; ++j)
      if (j < nnext) load_row_regs<C, NRC>(row_src(yl + ky0 + kyn + j), chunks, gin.x, nrow[j]);
    for (int ky = ky0; ky < ky0 + kyn; ++ky) {
      if (ky >= wk_lo && ky <= wk_hi) {
        int aoff[AM];
#pragma unroll
        for (int mb = 0; mb < AM; ++mb) aoff[mb] = ((ypos[mb] + ky) % RING) * pitch;
        // the MFMAs of tap (ky, kx) with its B fragments
        // A fragments of tap kx (every k-step, every position block) into registers: all of a tap's
        // reads are issued before its first MFMA (round 5's loop read one fragment, waited for it and
        // ran its MFMA, one LDS latency per MFMA: profiles/r06c_conv1_isa.txt)
        auto read_a = [&](int kx, bf16x8 (&a)[KSTEPS][AM]) {
          int abase[AM];  // the lane's column of each block, or the zero column outside the tensor (PAD)
#pragma unroll
          for (int mb = 0; mb < AM; ++mb) {
            const int col = xcol[mb] + kx * dx;
            if constexpr (PL) {  // chunk j = 2 s + kh of the column: plane j
              abase[mb] = aoff[mb] + 16 * (!PAD || (unsigned)col < (unsigned)W ? col : W) + kh * plane;
            } else {
              abase[mb] = (!PAD || (unsigned)col < (unsigned)W ? aoff[mb] + cell_off<C>(col) : zero_off) + kh * 16;
            }
          }
#pragma unroll
          for (int s = 0; s < KSTEPS; ++s)
#pragma unroll
            for (int mb = 0; mb < AM; ++mb)
              a[s][mb] = *(const bf16x8*)(lds + abase[mb] + (PL ? s * (M::KS / 8) * plane : s * M::KS * 2));
        };
        auto mma_tap = [&](const bf16x8 (&a)[KSTEPS][AM], const bf16x8 (&bt)[AN][KSTEPS]) {
#pragma unroll
          for (int s = 0; s < KSTEPS; ++s)
#pragma unroll
            for (int mb = 0; mb < AM; ++mb)
#pragma unroll
              for (int nb = 0; nb < AN; ++nb) acc[mb][nb] = M::mma(a[s][mb], bt[nb][s], acc[mb][nb]);
        };
        auto tap = [&](int kx, const bf16x8 (&bt)[AN][KSTEPS]) {
          bf16x8 a[KSTEPS][AM];
          read_a(kx, a);
          mma_tap(a, bt);
        };
        // two A register sets where they fit beside the rest: accumulators + two A sets + two B sets
        // within 168 of the 256 registers (the 64-channel padded data-gradient form, 16 A fragments a
        // tap, and conv2's two channel blocks, 128 accumulator registers, spilled with two A sets)
        constexpr bool kAAhead =
            AM * AN * (MS * MS / 64) + 2 * 4 * KSTEPS * AM + 2 * 4 * AN * KSTEPS <= 168;
        auto pin = [] {
          if constexpr (PIN) __builtin_amdgcn_sched_barrier(0);
        };
        if constexpr (kBAhead == 2 && kAAhead) {
          // two taps per trip, B in two register sets that swap roles without copies: the next tap's
          // fragments are requested before this tap's MFMAs and waited for a whole tap later; A the
          // same way within the kernel row (the next tap's reads in flight during this tap's MFMAs)
          bf16x8 a0[KSTEPS][AM], a1[KSTEPS][AM];
          int kx = 0;
          if (KW > 1) read_a(0, a0);
          for (; kx + 1 < KW; kx += 2) {
            load_b(ky * KW + kx + 1, bnx);
            read_a(kx + 1, a1);
            pin();
            mma_tap(a0, bcur);
            pin();
            load_b(ky * KW + kx + 2, bcur);
            if (kx + 2 < KW) read_a(kx + 2, a0);
            pin();
            mma_tap(a1, bnx);
            pin();
          }
          if (kx < KW) {  // odd KW: the last tap, then its successor's fragments back into bcur
            load_b(ky * KW + kx + 1, bnx);
            tap(kx, bcur);
#pragma unroll
            for (int nb = 0; nb < AN; ++nb)
#pragma unroll
              for (int s = 0; s < KSTEPS; ++s) bcur[nb][s] = bnx[nb][s];
          }
        } else if constexpr (kBAhead == 2) {
          int kx = 0;
          for (; kx + 1 < KW; kx += 2) {
            bf16x8 a[KSTEPS][AM];
            load_b(ky * KW + kx + 1, bnx);
            read_a(kx, a);
            pin();
            mma_tap(a, bcur);
            pin();
            load_b(ky * KW + kx + 2, bcur);
            read_a(kx + 1, a);
            pin();
            mma_tap(a, bnx);
            pin();
          }
          if (kx < KW) {
            load_b(ky * KW + kx + 1, bnx);
            tap(kx, bcur);
#pragma unroll
            for (int nb = 0; nb < AN; ++nb)
#pragma unroll
              for (int s = 0; s < KSTEPS; ++s) bcur[nb][s] = bnx[nb][s];
          }
        } else {
          for (int kx = 0; kx < KW; ++kx) {
            bf16x8 bnext[AN][KSTEPS];
            bf16x8 a[KSTEPS][AM];
            load_b(ky * KW + kx + 1, bnext);
            read_a(kx, a);
            pin();
            mma_tap(a, bcur);
            pin();
#pragma unroll
            for (int nb = 0; nb < AN; ++nb)
#pragma unroll
              for (int s = 0; s < KSTEPS; ++s) bcur[nb][s] = bnext[nb][s];
          }
        }
      }
    }
    if constexpr (KYS == 1) {
      if (nnext > 0) store_row(lds + ((yl + ky0 + 1) % RING) * pitch, nrow[0]);
      __syncthreads();
    } else {
      __syncthreads();  // every wave done with the rows the new ones replace
#pragma unroll
      for (int j = 0; j < KYS; ++j)
        if (j < nnext) store_row(lds + ((yl + ky0 + kyn + j) % RING) * pitch, nrow[j]);
      __syncthreads();
    }
  }

  // epilogue: C/D column = lane & (MS - 1) (channel), row = Mfma<MS>::row(i, kh) (position)
  const bool relu = flags & FFMP_CONV_RELU, out_bf16 = flags & FFMP_CONV_OUT_BF16;
#pragma unroll
  for (int nb = 0; nb < AN; ++nb) {
    const int n = nb * MS + r;
    const float bn = bias ? bias[n] : 0.f;
#pragma unroll
    for (int mb = 0; mb < AM; ++mb) {
      const int mbase = pw0 + mb * MS;
#pragma unroll
      for (int i = 0; i < M::NACC; ++i) {
        const int m = mbase + M::row(i, kh);
        if (m >= P) continue;
        float v = acc[mb][nb][i] + bn;
        if (relu) v = fmaxf(v, 0.f);
        const size_t o = ((size_t)b * P + m) * N + n;
        if (out_bf16)
          ((__bf16*)y)[o] = (__bf16)v;
        else
          ((float*)y)[o] = v;
      }
    }
  }
}

// The row-ring forward with each tap's B operand shared through LDS (FFMP_TUNE_CONV_LB): the
// workgroup's 256 threads load the next tap's weights (N x C x 2 bytes = 4 KiB at conv2's shape, one
// 16-byte chunk per thread) into registers during the current tap and write them, in fragment order,
// into the other of two LDS tap buffers; one barrier per tap publishes them, and every wave reads its
// B fragments from LDS (1 KiB contiguous per fragment: conflict-free ds_read_b128) instead of from
// L1/L2 — a quarter of the weight requests, 4 staging registers instead of a 16-register next-tap
// set.  The ring holds exactly the tile's span of rows (no spare slot): the next row is written
// between two barriers at the end of each kernel row.  Unpadded (pad 0), plain or fragment-order
// weights, C * N * 2 == 4096 bytes per tap (256 chunks).
template <int C, int NB, int MBW, bool WF>
__global__ __launch_bounds__(256, FFMP_CONV_FWD_OCC) void conv_fwd_lb_kernel(const __bf16* __restrict__ x,
                                                                             const __bf16* __restrict__ w,
                                                                             const float* __restrict__ bias,
                                                                             void* __restrict__ y, int H, int W, int KH,
                                                                             int KW, int dx, int RING, int flags) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  constexpr int N = NB * 32;
  constexpr int PT = kWaves * MBW * 32;
  constexpr int TAPB = N * C * 2;  // bytes of one tap's weights
  static_assert(TAPB == 4096, "one 16-byte chunk per thread per tap");
  const int Ho = H - KH + 1, Wo = W - (KW - 1) * dx;
  const int b = blockIdx.y;
  const int P = Ho * Wo;
  const int p0 = blockIdx.x * PT;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  const int rowbytes = W * C * 2;
  const int pitch = lds_pitch<C>(W);
  const int chunks = rowbytes / 16;
  const int2 gin = in_geom<C>(W, dx, flags);
  char* bbuf = lds + RING * pitch;  // two tap buffers after the ring
  const int yf = p0 / Wo;
  const int yl = min(P - 1, p0 + PT - 1) / Wo;
  const char* xb = (const char*)x + (size_t)b * H * gin.y;
  const int pw0 = p0 + wave * MBW * 32;
  int ypos[MBW], xcol[MBW];
#pragma unroll
  for (int mb = 0; mb < MBW; ++mb) {
    const int m = min(pw0 + mb * 32 + r, P - 1);
    ypos[mb] = m / Wo;
    xcol[mb] = m - ypos[mb] * Wo;
  }
  // this thread's chunk of a tap: global chunk q = threadIdx.x -> its fragment-order LDS offset
  const int q = threadIdx.x;
  int bdst;
  if constexpr (WF) {
    bdst = q * 16;
  } else {  // plain [n][c]: n = q / (C / 8), 8 channels c0 = (q % (C / 8)) * 8
    const int n = q / (C / 8), c0 = (q % (C / 8)) * 8;
    bdst = ((((n >> 5) * (C / 16) + (c0 >> 4)) * 2 + ((c0 >> 3) & 1)) * 256 + (n & 31) * 8) * 2;
  }
  const char* wsrc = (const char*)w + q * 16;
  for (int row = yf; row <= yl; ++row) {
    uint4 buf[4];
    load_row_regs<C>(xb + (size_t)row * gin.y, chunks, gin.x, buf);
    store_row_lds<C>(lds + (row % RING) * pitch, chunks, buf);
  }
  *(uint4*)(bbuf + bdst) = *(const uint4*)wsrc;  // tap 0 into buffer 0
  __syncthreads();

  f32x16 acc[MBW][NB];
#pragma unroll
  for (int mb = 0; mb < MBW; ++mb)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) acc[mb][nb] = f32x16{};
  const int ntaps = KH * KW;
  int t = 0;
  for (int ky = 0; ky < KH; ++ky) {
    uint4 nrow[4];
    const bool more = ky + 1 < KH;
    if (more) load_row_regs<C>(xb + (size_t)(yl + ky + 1) * gin.y, chunks, gin.x, nrow);
    int aoff[MBW];
#pragma unroll
    for (int mb = 0; mb < MBW; ++mb) aoff[mb] = ((ypos[mb] + ky) % RING) * pitch;
    for (int kx = 0; kx < KW; ++kx, ++t) {
      const bool bnext = t + 1 < ntaps;
      uint4 stage = uint4{0u, 0u, 0u, 0u};
      if (bnext) stage = *(const uint4*)(wsrc + (size_t)(t + 1) * TAPB);
      const char* bt = bbuf + (t & 1) * TAPB;
      bf16x8 bf[NB][C / 16];
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
#pragma unroll
        for (int s2 = 0; s2 < C / 16; ++s2)
          bf[nb][s2] = *(const bf16x8*)(bt + (((nb * (C / 16) + s2) * 2 + h) * 256 + r * 8) * 2);
      int abase[MBW];
#pragma unroll
      for (int mb = 0; mb < MBW; ++mb) abase[mb] = aoff[mb] + cell_off<C>(xcol[mb] + kx * dx) + h * 16;
#pragma unroll
      for (int s2 = 0; s2 < C / 16; ++s2) {
        bf16x8 a[MBW];
#pragma unroll
        for (int mb = 0; mb < MBW; ++mb) a[mb] = *(const bf16x8*)(lds + abase[mb] + s2 * 32);
#pragma unroll
        for (int mb = 0; mb < MBW; ++mb)
#pragma unroll
          for (int nb = 0; nb < NB; ++nb)
            acc[mb][nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[mb], bf[nb][s2], acc[mb][nb], 0, 0, 0);
      }
      if (bnext) *(uint4*)(bbuf + ((t + 1) & 1) * TAPB + bdst) = stage;
      __syncthreads();  // tap t + 1's weights published; tap t's buffer free again
    }
    if (more) {  // the slot of row yf + ky (no wave reads it any more) takes row yl + ky + 1
      store_row_lds<C>(lds + ((yl + ky + 1) % RING) * pitch, chunks, nrow);
      __syncthreads();
    }
  }

  const bool relu = flags & FFMP_CONV_RELU, out_bf16 = flags & FFMP_CONV_OUT_BF16;
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const int n = nb * 32 + r;
    const float bn = bias ? bias[n] : 0.f;
#pragma unroll
    for (int mb = 0; mb < MBW; ++mb) {
      const int mbase = pw0 + mb * 32;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int m = mbase + (i & 3) + 8 * (i >> 2) + 4 * h;
        if (m >= P) continue;
        float v = acc[mb][nb][i] + bn;
        if (relu) v = fmaxf(v, 0.f);
        const size_t o = ((size_t)b * P + m) * N + n;
        if (out_bf16)
          ((__bf16*)y)[o] = (__bf16)v;
        else
          ((float*)y)[o] = v;
      }
    }
  }
}

// Small images (the reference Network's conv3 / conv4: 8 x 8 kernels over 38^2 .. 17^2 maps, and
// their data gradients): a 512-position tile wastes most of its positions on a 10^2 or 17^2
// image, and 128-position tiles leave each wave one 32-position block (every B fragment used
// once).  Here a workgroup owns 128 positions x all N channels and its 4 waves split the K loop
// instead (wave w takes kernel rows ky = w, w + 4, ...), each holding all 4 position blocks x NB
// channel blocks; the input window of the tile (all its rows for every ky) is staged in LDS once,
// and the 4 partial accumulators are summed through LDS in the epilogue.
template <int C, int NB, bool PAD, bool WF, int MS = 32>
__global__ __launch_bounds__(256, 2) void conv_small_kernel(const __bf16* __restrict__ x, const __bf16* __restrict__ w,
                                                            const float* __restrict__ bias, void* __restrict__ y,
                                                            int H, int W, int KH, int KW, int pad, int dx, int flags) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  using M = Mfma<MS>;
  constexpr int N = NB * 32, PT = 128;
  constexpr int AM = PT / MS, AN = N / MS;  // MFMA blocks per wave: all 128 positions x all N channels
  constexpr int KSTEPS = C / M::KS;
  const int Ho = H + 2 * pad - KH + 1, Wo = W + 2 * pad - (KW - 1) * dx;
  const int b = blockIdx.y;
  const int P = Ho * Wo;
  const int p0 = blockIdx.x * PT;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & (MS - 1), kh = lane / MS;
  const int rowbytes = W * C * 2;
  const int pitch = lds_pitch<C>(W);  // padded row images (cell_off)
  const int2 gin = in_geom<C>(W, dx, flags);
  const int chunks = rowbytes / 16;
  const int yf = p0 / Wo;
  const int yl = min(P - 1, p0 + PT - 1) / Wo;
  const char* xb = (const char*)x + (size_t)b * H * gin.y;
  const int ky_lo = max(0, pad - yl), ky_hi = min(KH - 1, pad + H - 1 - yf);
  const int zero_off = (yl + ky_hi - yf - ky_lo + 1) * pitch;  // a zero column after the window

  // the window: logical rows [yf + ky_lo, yl + ky_hi], slot = row - yf - ky_lo
  for (int row = yf + ky_lo; row <= yl + ky_hi; ++row) {
    const int real = row - pad;
    const char* src = (real >= 0 && real < H) ? xb + (size_t)real * gin.y : nullptr;
    for (int q0 = 0; q0 < chunks; q0 += 1024) {
      uint4 buf[4];
      load_row_regs<C>(src ? src + (size_t)(q0 / (C / 8)) * gin.x : nullptr, chunks - q0, gin.x, buf);
      store_row_lds<C>(lds + (row - yf - ky_lo) * pitch + cell_off<C>(q0 / (C / 8)), chunks - q0, buf);
    }
  }
  if (PAD && threadIdx.x < C / 8) *(uint4*)(lds + zero_off + 16 * threadIdx.x) = uint4{0u, 0u, 0u, 0u};
  int ypos[AM], xcol[AM];
#pragma unroll
  for (int mb = 0; mb < AM; ++mb) {
    const int m = min(p0 + mb * MS + r, P - 1);
    ypos[mb] = m / Wo - yf - ky_lo;  // window slot of kernel row ky_lo
    xcol[mb] = m % Wo - pad;
  }
  __syncthreads();

  typename M::acc_t acc[AM][AN];
#pragma unroll
  for (int mb = 0; mb < AM; ++mb)
#pragma unroll
    for (int nb = 0; nb < AN; ++nb) acc[mb][nb] = typename M::acc_t{};

  for (int ky = ky_lo + wave; ky <= ky_hi; ky += kWaves) {
    int aoff[AM];
#pragma unroll
    for (int mb = 0; mb < AM; ++mb) aoff[mb] = (ypos[mb] + ky) * pitch;
    bf16x8 bcur[AN][KSTEPS];
#pragma unroll
    for (int nb = 0; nb < AN; ++nb)
#pragma unroll
      for (int s = 0; s < KSTEPS; ++s) bcur[nb][s] = load_bfrag_ms<C, NB, WF, MS>(w, ky * KW, nb, s, r, kh);
    for (int kx = 0; kx < KW; ++kx) {
      const int tn = ky * KW + min(kx + 1, KW - 1);
      bf16x8 bnext[AN][KSTEPS];
#pragma unroll
      for (int nb = 0; nb < AN; ++nb)
#pragma unroll
        for (int s = 0; s < KSTEPS; ++s) bnext[nb][s] = load_bfrag_ms<C, NB, WF, MS>(w, tn, nb, s, r, kh);
      int abase[AM];
#pragma unroll
      for (int mb = 0; mb < AM; ++mb) {
        const int col = xcol[mb] + kx * dx;
        abase[mb] = (!PAD || (unsigned)col < (unsigned)W ? aoff[mb] + cell_off<C>(col) : zero_off) + kh * 16;
      }
#pragma unroll
      for (int s = 0; s < KSTEPS; ++s) {
        bf16x8 a[AM];
#pragma unroll
        for (int mb = 0; mb < AM; ++mb) a[mb] = *(const bf16x8*)(lds + abase[mb] + s * M::KS * 2);
#pragma unroll
        for (int mb = 0; mb < AM; ++mb)
#pragma unroll
          for (int nb = 0; nb < AN; ++nb) acc[mb][nb] = M::mma(a[mb], bcur[nb][s], acc[mb][nb]);
      }
#pragma unroll
      for (int nb = 0; nb < AN; ++nb)
#pragma unroll
        for (int s = 0; s < KSTEPS; ++s) bcur[nb][s] = bnext[nb][s];
    }
  }

  // sum the 4 waves' partials through LDS, one channel block at a time: red[wave][mb][i][lane]
  const bool relu = flags & FFMP_CONV_RELU, out_bf16 = flags & FFMP_CONV_OUT_BF16;
  float* red = (float*)lds;
  constexpr int E = AM * M::NACC * 64;  // entries per wave (= 4 * 16 * 64 for either shape)
#pragma unroll
  for (int nb = 0; nb < AN; ++nb) {
    __syncthreads();  // the window (nb = 0) or the previous block's sums are no longer read
#pragma unroll
    for (int mb = 0; mb < AM; ++mb)
#pragma unroll
      for (int i = 0; i < M::NACC; ++i) red[wave * E + (mb * M::NACC + i) * 64 + lane] = acc[mb][nb][i];
    __syncthreads();
    for (int e = threadIdx.x; e < E; e += 256) {
      const int ln = e & 63, i = (e >> 6) % M::NACC, mb = (e >> 6) / M::NACC;
      const int m = p0 + mb * MS + M::row(i, ln / MS);
      if (m >= P) continue;
      const int n = nb * MS + (ln & (MS - 1));
      float v = red[e] + red[E + e] + red[2 * E + e] + red[3 * E + e] + (bias ? bias[n] : 0.f);
      if (relu) v = fmaxf(v, 0.f);
      const size_t o = ((size_t)b * P + m) * N + n;
      if (out_bf16)
        ((__bf16*)y)[o] = (__bf16)v;
      else
        ((float*)y)[o] = v;
    }
  }
}

constexpr size_t kSmallRedBytes = 4 * 4 * 16 * 64 * sizeof(float);  // conv_small_kernel's reduction: 64 KiB

// LDS bytes of conv_small_kernel's window for this shape (a 128-position tile's rows + KH - 1)
size_t small_window_bytes(int Wo, int KH, int W, int C) {
  const int pitch = C == 64 ? lds_pitch<64>(W) : lds_pitch<32>(W);
  return (size_t)((128 + Wo - 1) / Wo + 1 + KH - 1) * pitch + C * 2;  // + the zero column
}

template <int C, int NB, bool PAD, bool WF>
int launch_small(const void* x, const void* w, const float* bias, void* y, int B, int H, int W, int KH, int KW, int pad,
                 int dx, int flags, hipStream_t s) {
  const int Ho = H + 2 * pad - KH + 1, Wo = W + 2 * pad - (KW - 1) * dx;
  const size_t lds = std::max(small_window_bytes(Wo, KH, W, C), kSmallRedBytes);
  const dim3 grid((Ho * Wo + 127) / 128, B);
  if (t_conv_dry) return FFMP_OK;
  // MFMA shape: 16x16x32 for the padded (data-gradient) form — conv3's 0.199 -> 0.192 ms, conv4's 0.145 ->
  // 0.137 at B = 256 — 32x32x16 for the forwards (conv3 0.153 vs 0.162; profiles/r06j_conv_ab_small_ms16.txt)
  if (ffmp_detail::mfma_for(PAD ? 16 : 32) == 16)
    hipLaunchKernelGGL((conv_small_kernel<C, NB, PAD, WF, 16>), grid, dim3(256), lds, s, (const __bf16*)x,
                       (const __bf16*)w, bias, y, H, W, KH, KW, pad, dx, flags);
  else
    hipLaunchKernelGGL((conv_small_kernel<C, NB, PAD, WF, 32>), grid, dim3(256), lds, s, (const __bf16*)x,
                       (const __bf16*)w, bias, y, H, W, KH, KW, pad, dx, flags);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(FFMP_E_HIP, "ffmp_conv2d launch: %s", hipGetErrorString(e));
  return FFMP_OK;
}

// positions per workgroup: 512 (MBW 4), 384, 256 or 128.  First the largest tile (the most reuse of
// each B fragment) whose rounding of an image's positions costs at most 10 % more than the tightest
// and whose ring leaves room for two workgroups per CU.  Then, when that is the 512-position tile, a
// grid-fill check against the 384-position one: B * ceil(P / PT) workgroups in rounds of `slots`
// (CUs x the kernel's occupancy at that tile's LDS); a round costs PT x its workgroups per CU, a
// partial last round with a fraction f of the slots 0.3 + 0.7 f of a full one (its CUs run fewer
// waves, at a lower rate), and the 384-position tile's per-position rate is 0.96 of the 512's (less
// reuse; profiles/r06e_conv_ab*.txt).  Conv2 at B = 256 (1,444 positions, 2 per CU on 256 CUs): 512
// tiles = 768 workgroups = 1.5 rounds, 384 tiles = 1,024 = 2 full rounds: 1.19 vs 1.23 ms; at B =
// 1,024 both fill their rounds and the 512 tile stays (4.50 vs 4.70 ms).  Never changes results
// (each position's sum runs over the same taps in the same order).
int pick_mbw(int P, int Wo, size_t slotbytes, int B, int slots4, int slots3) {
  static const int forced_env = [] {  // FFMP_CONV_MBW = 1 / 2 / 3 / 4: a probe knob (tools/conv_variants.py)
    const char* v = getenv("FFMP_CONV_MBW");
    const int m = v ? atoi(v) : 0;
    return (m >= 1 && m <= 4) ? m : 0;
  }();
  const int forced = ffmp_detail::g_conv_mbw ? ffmp_detail::g_conv_mbw : forced_env;
  if (forced) return forced;
  long padded[3], least = -1;
  const int mbws[3] = {4, 2, 1};
  for (int i = 0; i < 3; ++i) {
    const int pt = kWaves * mbws[i] * 32;
    padded[i] = (long)((P + pt - 1) / pt) * pt;
    if (least < 0 || padded[i] < least) least = padded[i];
  }
  int pick = 1;
  for (int i = 0; i < 3; ++i) {
    const int pt = kWaves * mbws[i] * 32;
    const size_t ring = (size_t)((pt + Wo - 1) / Wo + 2) * slotbytes;
    if ((ring <= 80 * 1024 || mbws[i] == 1) && padded[i] * 10 <= least * 11) {
      pick = mbws[i];
      break;
    }
  }
  if (pick != 4 || slots4 <= 0 || slots3 <= 0) return pick;
  auto cost = [&](int mbw, int slots, double eff) {
    const long pt = kWaves * mbw * 32;
    const double wgs = (double)B * (double)((P + pt - 1) / pt), r = wgs / slots, full = (double)(long)r, f = r - full;
    return (full + (f > 0 ? 0.3 + 0.7 * f : 0.0)) * (double)pt * (double)slots / eff;
  };
  return cost(3, slots3, 0.96) < cost(4, slots4, 1.0) ? 3 : 4;
}

// CUs of the current device (256 on MI355X; that, when there is none: the dry-run shape checks)
int device_cus() {
  static std::mutex mu;
  static std::map<int, int> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(dev);
  if (it != cache.end()) return it->second;
  int n = 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  cache[dev] = n;
  return n;
}

// workgroups of a kernel resident per CU at `lds` bytes of dynamic LDS (2 when the runtime cannot say)
int wgs_per_cu(const void* fn, size_t lds) {
  static std::mutex mu;
  static std::map<std::pair<const void*, size_t>, int> cache;
  std::lock_guard<std::mutex> lk(mu);
  const auto key = std::make_pair(fn, lds);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, 256, lds) != hipSuccess || n <= 0) {
    (void)hipGetLastError();
    n = 2;
  }
  cache[key] = n;
  return n;
}

// the row-ring forward on planar slots (FFMP_TUNE_CONV_PLANAR): 32x32x16, one kernel row per ring step,
// not with the conv2-shaped pinned-schedule variants (FFMP_TUNE_CONV_BA2) or B through LDS
template <int C, int NB, bool PAD>
bool use_planar(int chunks) {
  if (ffmp_detail::g_conv_planar != 1) return false;
  if (ffmp_detail::mfma_for(32) != 32 || ffmp_detail::g_conv_kys > 1 || ffmp_detail::g_conv_lb == 1) return false;
  if (C == 32 && NB == 2 && !PAD && (ffmp_detail::g_conv_ba2 == 2 || (ffmp_detail::g_conv_ba2 == 1 && chunks <= 512)))
    return false;
  return true;
}

template <int C, int NB, int MBW, bool PAD, bool WF>
int launch_fwd_mbw(const void* x, const void* w, const float* bias, void* y, int B, int H, int W, int KH, int KW,
                   int pad, int dx, int flags, hipStream_t s) {
  const int Ho = H + 2 * pad - KH + 1, Wo = W + 2 * pad - (KW - 1) * dx;
  constexpr int PT = kWaves * MBW * 32;
  const int span = (PT + Wo - 1) / Wo + 1;  // input rows a tile reads for one ky
  const bool planar = use_planar<C, NB, PAD>((W * C * 2) / 16);
  const size_t pitch = planar ? (size_t)planar_pitch<C>(W, Wo, PAD) : (size_t)lds_pitch<C>(W);
  // kernel rows per ring step (FFMP_TUNE_CONV_KYS; 0 = default 1).  Built for the one-channel-block
  // layers (conv1 carries 16 MFMAs per wave per kernel row and parks 0.43 of its wave cycles,
  // profiles/r05e_conv_pmc.txt) but measured slower: conv1 0.269 ms at 1 row per step, 0.296 at 2 and
  // 4; conv2 1.28 / 1.27 / 1.51 ms (profiles/r06b_conv_ab.txt) — kept as a probe knob, default 1
  auto ring_of = [&](int k) { return k == 1 ? span + 1 : span + k - 1; };
  auto lds_of = [&](int k) { return (size_t)ring_of(k) * pitch + C * 2; };  // + the zero column
  int kys = ffmp_detail::g_conv_kys;
  if (kys == 0) kys = 1;
  if (kys != 1 && kys != 2 && kys != 4) kys = 1;
  const int ring = ring_of(kys);
  const size_t lds = lds_of(kys);
  if (lds > 160 * 1024)
    return fail(FFMP_E_ARG, "ffmp_conv2d: a ring of %d input rows (%zu bytes) exceeds the 160 KiB LDS", ring, lds);
  if ((W * C * 2) / 16 > 4 * 256) return fail(FFMP_E_ARG, "ffmp_conv2d: input rows wider than 16 KiB");
  const dim3 grid((Ho * Wo + PT - 1) / PT, B);
  // B through LDS (FFMP_TUNE_CONV_LB): the unpadded 4 KiB-per-tap layers, ring = span + two tap buffers
  if constexpr (C * NB * 32 * 2 == 4096) {
    const size_t lds_lb = (size_t)span * lds_pitch<C>(W) + 2 * 4096;
    if (!PAD && !planar && ffmp_detail::g_conv_lb == 1 && lds_lb <= 80 * 1024) {
      if (t_conv_dry) return FFMP_OK;
      hipLaunchKernelGGL((conv_fwd_lb_kernel<C, NB, MBW, WF>), grid, dim3(256), lds_lb, s, (const __bf16*)x,
                         (const __bf16*)w, bias, y, H, W, KH, KW, dx, span, flags);
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) return fail(FFMP_E_HIP, "ffmp_conv2d launch: %s", hipGetErrorString(e));
      return FFMP_OK;
    }
  }
  if (t_conv_dry) return FFMP_OK;
  const int chunks = (W * C * 2) / 16;
  auto go = [&](auto MS_, auto KYS_) {
    constexpr int kMS = decltype(MS_)::value, kKYS = decltype(KYS_)::value;
    if constexpr (kMS == 32 && kKYS == 1) {
      if (ffmp_detail::g_conv_pin == 1 && !planar) {
        hipLaunchKernelGGL((conv_fwd_kernel<C, NB, MBW, PAD, WF, 32, 1, 4, 0, true, false>), grid, dim3(256), lds, s,
                           (const __bf16*)x, (const __bf16*)w, bias, y, H, W, KH, KW, pad, dx, ring, flags);
        return;
      }
      if (planar) {
        hipLaunchKernelGGL((conv_fwd_kernel<C, NB, MBW, PAD, WF, 32, 1, 4, 0, false, true>), grid, dim3(256), lds, s,
                           (const __bf16*)x, (const __bf16*)w, bias, y, H, W, KH, KW, pad, dx, ring, flags);
        return;
      }
    }
    // one channel block, several kernel rows per ring step (FFMP_TUNE_CONV_KYS 2 / 4): the next rows in
    // 2 registers per thread where they fit (rows up to 8 KiB: the folded conv1's 5.3 KiB)
    if constexpr (NB == 1 && !PAD && kMS == 32 && kKYS > 1) {
      if (chunks <= 512) {
        hipLaunchKernelGGL((conv_fwd_kernel<C, NB, MBW, PAD, WF, 32, kKYS, 2>), grid, dim3(256), lds, s,
                           (const __bf16*)x, (const __bf16*)w, bias, y, H, W, KH, KW, pad, dx, ring, flags);
        return;
      }
    }
    // conv2's shape (32 -> 64, unpadded): the pinned-schedule variants (FFMP_TUNE_CONV_BA2: 1 = B two
    // taps ahead with rows in 2 registers where the row fits, 2 = B one tap ahead)
    if constexpr (C == 32 && NB == 2 && !PAD && kMS == 32 && kKYS == 1) {
      const int ba2 = ffmp_detail::g_conv_ba2;
      if (chunks <= 512 && ba2 == 1) {
        hipLaunchKernelGGL((conv_fwd_kernel<C, NB, MBW, PAD, WF, 32, 1, 2, 2, true>), grid, dim3(256), lds, s,
                           (const __bf16*)x, (const __bf16*)w, bias, y, H, W, KH, KW, pad, dx, ring, flags);
        return;
      }
      if (ba2 == 2) {
        hipLaunchKernelGGL((conv_fwd_kernel<C, NB, MBW, PAD, WF, 32, 1, 4, 1, true>), grid, dim3(256), lds, s,
                           (const __bf16*)x, (const __bf16*)w, bias, y, H, W, KH, KW, pad, dx, ring, flags);
        return;
      }
    }
    hipLaunchKernelGGL((conv_fwd_kernel<C, NB, MBW, PAD, WF, kMS, kKYS>), grid, dim3(256), lds, s, (const __bf16*)x,
                       (const __bf16*)w, bias, y, H, W, KH, KW, pad, dx, ring, flags);
  };
  auto with_ms = [&](auto KYS_) {
    if (ffmp_detail::mfma_for(32) == 16) go(std::integral_constant<int, 16>{}, KYS_);
    else go(std::integral_constant<int, 32>{}, KYS_);
  };
  if constexpr (MBW == 3) {  // built for the default launch only (pick_mbw offers it for no other)
    go(std::integral_constant<int, 32>{}, std::integral_constant<int, 1>{});
  } else if constexpr (NB == 1) {
    if (kys == 4) with_ms(std::integral_constant<int, 4>{});
    else if (kys == 2) with_ms(std::integral_constant<int, 2>{});
    else with_ms(std::integral_constant<int, 1>{});
  } else {
    if (kys == 2) with_ms(std::integral_constant<int, 2>{});
    else with_ms(std::integral_constant<int, 1>{});
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(FFMP_E_HIP, "ffmp_conv2d launch: %s", hipGetErrorString(e));
  return FFMP_OK;
}

// the default launch of launch_fwd_mbw (KYS 1, the configured MFMA shape): workgroups per CU, 0 when
// its ring exceeds the LDS
template <int C, int NB, int MBW, bool PAD, bool WF>
int fwd_occupancy(int W, int Wo) {
  constexpr int PT = kWaves * MBW * 32;
  const bool planar = use_planar<C, NB, PAD>((W * C * 2) / 16);
  const size_t lds = (size_t)((PT + Wo - 1) / Wo + 2) * (planar ? planar_pitch<C>(W, Wo, PAD) : lds_pitch<C>(W)) + C * 2;
  if (lds > 160 * 1024) return 0;
  if (planar) return wgs_per_cu((const void*)conv_fwd_kernel<C, NB, MBW, PAD, WF, 32, 1, 4, 0, false, true>, lds);
  if constexpr (MBW == 3) {  // the default launch only (32x32x16, one kernel row per ring step)
    if (ffmp_detail::mfma_for(32) != 32 || ffmp_detail::g_conv_kys > 1) return 0;
    return wgs_per_cu((const void*)conv_fwd_kernel<C, NB, MBW, PAD, WF, 32, 1>, lds);
  } else {
    const void* fn = ffmp_detail::mfma_for(32) == 16 ? (const void*)conv_fwd_kernel<C, NB, MBW, PAD, WF, 16, 1>
                                                     : (const void*)conv_fwd_kernel<C, NB, MBW, PAD, WF, 32, 1>;
    return wgs_per_cu(fn, lds);
  }
}

template <int C, int NB, bool PAD, bool WF>
int launch_fwd_wf(const void* x, const void* w, const float* bias, void* y, int B, int H, int W, int KH, int KW, int pad,
               int dx, int flags, hipStream_t s) {
  const int Ho = H + 2 * pad - KH + 1, Wo = W + 2 * pad - (KW - 1) * dx;
  // small images with a kernel deep enough to split over the waves: conv_small_kernel
  if (Ho * Wo <= 2048 && KH >= 4 && small_window_bytes(Wo, KH, W, C) <= 76 * 1024 && (W * C * 2) % 16 == 0)
    return launch_small<C, NB, PAD, WF>(x, w, bias, y, B, H, W, KH, KW, pad, dx, flags, s);
  int slots4 = 0, slots3 = 0;  // 0: no grid-fill check (the dry-run shape checks, one channel block)
  if (!t_conv_dry) {
    const int cus = device_cus();
    if constexpr (NB == 2) {  // measured for the two-channel-block layers only (conv2's forward);
      // the folded conv1 (one block) ran 8 % slower on 384 tiles at 2 workgroups per CU than on 512
      // at 3, which the model above does not see
      slots4 = cus * fwd_occupancy<C, NB, 4, PAD, WF>(W, Wo);
      slots3 = cus * fwd_occupancy<C, NB, 3, PAD, WF>(W, Wo);
    }
  }
  switch (pick_mbw(Ho * Wo, Wo, (size_t)lds_pitch<C>(W), B, slots4, slots3)) {
    case 4: return launch_fwd_mbw<C, NB, 4, PAD, WF>(x, w, bias, y, B, H, W, KH, KW, pad, dx, flags, s);
    case 3: return launch_fwd_mbw<C, NB, 3, PAD, WF>(x, w, bias, y, B, H, W, KH, KW, pad, dx, flags, s);
    case 2: return launch_fwd_mbw<C, NB, 2, PAD, WF>(x, w, bias, y, B, H, W, KH, KW, pad, dx, flags, s);
    default: return launch_fwd_mbw<C, NB, 1, PAD, WF>(x, w, bias, y, B, H, W, KH, KW, pad, dx, flags, s);
  }
}

template <int C, int NB, bool PAD>
int launch_fwd(const void* x, const void* w, const float* bias, void* y, int B, int H, int W, int KH, int KW, int pad,
               int dx, int flags, hipStream_t s) {
  if (flags & FFMP_CONV_W_FRAG) return launch_fwd_wf<C, NB, PAD, true>(x, w, bias, y, B, H, W, KH, KW, pad, dx, flags, s);
  return launch_fwd_wf<C, NB, PAD, false>(x, w, bias, y, B, H, W, KH, KW, pad, dx, flags, s);
}

// ------------------------------------------------------------------ weight gradient
// dW[tap][n][c] = sum_p g[p][n] * x[p + tap][c]: per tap a GEMM over positions, M = n (the output
// gradient g, NHWC [B][Ho][Wo][N]), N = c (the saved input x, NHWC [B][H][W][C]), K = positions.
// Both MFMA operands need positions along k, i.e. channel COLUMNS of the NHWC row images: they are
// read with ds_read_b64_tr_b16 (per 16 lanes, 4 image rows x 16 columns delivered column-major),
// lane (r, h) of the 32x32x16 operand getting image rows k0 + 8h .. +8 of its column r — from
// plain NHWC rows staged in LDS, no transposition pass.  128-byte image rows XOR their 16-byte
// chunk with ((row >> 1) & 1) << 2, so the 4 rows x 2 column halves of a 32-lane half cover all
// 64 banks.
//
// A workgroup owns TG = 4 * TW taps (a TKY x TKX rectangle of kernel rows / columns) and one chunk
// of the batch; wave w the taps [w * TW, (w + 1) * TW) of the rectangle, TW * NB * CB 32x32
// blocks (128 accumulators).  K runs over stages of R output rows of each sample (R * Wo
// positions, flattened, so no per-row padding): the stage's g rows and the x rows
// [y0 + kyA, y0 + R - 1 + kyA + TKY - 1] are copied to LDS (the next stage is loaded into
// registers while this one is consumed), then every wave walks the stage in k-steps of 16
// positions.  Each workgroup writes its taps' partial sums for its chunk of the batch:
// part[chunk][tap][n][c] (fp32); the caller sums over chunks.
__device__ __forceinline__ int swz128(int row) { return ((row >> 1) & 1) << 6; }  // bytes: chunk ^ 4

typedef short s16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ s16x4 tr_read(const char* p) {  // ds_read_b64_tr_b16 (8-byte aligned)
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)p);
}

constexpr int kWgradPieces = 12;  // 16-byte pieces of one stage per thread (<= 12 * 256: host check)

// Stage copies: one stage's g rows and x rows are contiguous byte ranges of g and x; piece k < gq
// comes from g, else from x; threads past the end re-read the last piece (no divergent loads).
// Written out in the kernel body: behind a helper taking the register array by reference,
// hipcc (ROCm 7.2) kept the array in scratch memory.
#define FFMP_WGRAD_LOAD1(i, gs, xs)                                                                  \
  {                                                                                                  \
    const int k = min((int)threadIdx.x + 256 * (i), gq + xq - 1);                                    \
    buf##i = *(const uint4*)(k < gq ? (gs) + 16 * (size_t)k : (xs) + 16 * (size_t)(k - gq));         \
  }
#define FFMP_WGRAD_LOAD(gs, xs)                                                                    \
  FFMP_WGRAD_LOAD1(0, gs, xs) FFMP_WGRAD_LOAD1(1, gs, xs) FFMP_WGRAD_LOAD1(2, gs, xs)              \
  FFMP_WGRAD_LOAD1(3, gs, xs) FFMP_WGRAD_LOAD1(4, gs, xs) FFMP_WGRAD_LOAD1(5, gs, xs)              \
  FFMP_WGRAD_LOAD1(6, gs, xs) FFMP_WGRAD_LOAD1(7, gs, xs) FFMP_WGRAD_LOAD1(8, gs, xs)              \
  FFMP_WGRAD_LOAD1(9, gs, xs) FFMP_WGRAD_LOAD1(10, gs, xs) FFMP_WGRAD_LOAD1(11, gs, xs)
// ... and into the LDS images (g rows: N * 2 bytes, x rows: C * 2 bytes; 128-byte rows swizzled)
#define FFMP_WGRAD_STORE1(i)                                                                         \
  {                                                                                                  \
    const int k = (int)threadIdx.x + 256 * (i);                                                      \
    const bool isg = k < gq;                                                                         \
    const int kk = isg ? k : k - gq, rb = isg ? N * 2 : C * 2, row = kk / (rb / 16);                 \
    const int off = (kk % (rb / 16)) * 16;                                                           \
    const bool sw = isg ? N == 64 : C == 64;                                                         \
    char* d = (isg ? gimg : ximg) + row * rb + (sw ? (off ^ swz128(row)) : off);                     \
    if (k < gq + xq) *(uint4*)d = buf##i;                                                            \
  }
#define FFMP_WGRAD_STORE()                                                                         \
  FFMP_WGRAD_STORE1(0) FFMP_WGRAD_STORE1(1) FFMP_WGRAD_STORE1(2) FFMP_WGRAD_STORE1(3)              \
  FFMP_WGRAD_STORE1(4) FFMP_WGRAD_STORE1(5) FFMP_WGRAD_STORE1(6) FFMP_WGRAD_STORE1(7)              \
  FFMP_WGRAD_STORE1(8) FFMP_WGRAD_STORE1(9) FFMP_WGRAD_STORE1(10) FFMP_WGRAD_STORE1(11)

// taps per wave of the 32 -> 64 weight gradient (conv2's): 8 (256 accumulators, one wave per SIMD)
// re-reads the stage images for half as many tap groups as 4: 1.73 vs 1.82-1.88 ms at B = 256
// (profiles/r04l_wgrad.txt)
#ifndef FFMP_WGRAD_TW_3264
#define FFMP_WGRAD_TW_3264 8
#endif
// 1: each k-step's operand reads are issued during the previous k-step's MFMAs (two register sets);
// -1: that for the 32 -> 64 kernel only (the smaller ones spill with it); 0 (default): not — the
// 32 -> 64 weight gradient ran 1.75-1.77 -> 1.82-1.83 ms with it (profiles/r04s_wgrad_prefetch.txt)
#ifndef FFMP_WGRAD_PREFETCH
#define FFMP_WGRAD_PREFETCH 0
#endif
// DMA (FFMP_TUNE_CONV_WGDMA): each stage is copied global -> LDS by LDS-DMA (global_load_lds_dwordx4,
// no staging registers) into one of TWO stage buffers, issued right after the stage's single barrier
// and landed during the previous stage's k-loop: no store phase, one barrier per stage instead of two,
// and the 48 staging registers free for the k-step prefetch (PF).  The LDS images stay as above: an
// LDS-DMA destination is wave-uniform base + 16 x lane, so each lane fetches the source chunk that
// the swizzled image holds at its linear position (the XOR is its own inverse).
template <int C, int N, int TW, int MS = 32, bool PF = false, bool DMA = false>
__global__ __launch_bounds__(256, (TW * (N / 32) * (C / 32) > 8 ? 1 : 2)) void conv_wgrad_kernel(const __bf16* __restrict__ g, const __bf16* __restrict__ x,
                                                            float* __restrict__ part, int B, int H, int W, int KH,
                                                            int KW, int dx, int TKY, int TKX, int R, int per_chunk) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  using M = Mfma<MS>;
  constexpr int AN = N / MS, AC = C / MS;  // MFMA blocks: output channels (rows) x input channels (columns)
  constexpr int KP = M::KS;                // positions per k-step (16 or 32)
  const int Ho = H - KH + 1, Wo = W - (KW - 1) * dx;
  const int groups_x = KW / TKX;
  const int kyA = (blockIdx.x / groups_x) * TKY, kxA = (blockIdx.x % groups_x) * TKX;
  const int b0 = blockIdx.y * per_chunk, b1 = min(B, b0 + per_chunk);
  // wave-uniform in a scalar register: the taps' offsets below are then scalar too (the compiler kept
  // them in 16 VGPRs and spent two VALU per operand read on them, profiles/r06c_wgrad_isa.txt)
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int fr = lane & (MS - 1), fk = lane / MS;       // operand row / k-chunk of 8 positions
  const int q = (lane & 15) >> 2, pp = lane & 3;        // tr-read: row q of 4, columns 4pp .. of 16
  const int gh = MS == 32 ? (lane >> 4) & 1 : 0;        // 32x32x16: the 16-column half of the 32
  const int grow = N * 2, xrowb = C * 2;             // image row bytes
  const int Pmax = R * Wo;                            // positions of a full stage
  const int SB = (Pmax + KP) * grow + (R + TKY - 1) * W * xrowb;  // one stage buffer (DMA: two)
  char* gimg = lds;
  char* ximg = lds + (Pmax + KP) * grow;              // g image + KP zero rows (k-steps past the stage end)

  // this wave's taps of the rectangle (the host makes the rectangle tile the kernel exactly);
  // the B image row of (position row pr, column pc) at tap t: (pr + dky[t]) * W + pc + dkx[t]
  int dky[TW], dkx[TW], toff[TW];
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    const int k = wave * TW + t;
    dky[t] = k / TKX;
    dkx[t] = (kxA + k % TKX) * dx;
    toff[t] = (dky[t] * W + dkx[t]) * (C * 2);  // byte offset of tap t's x row (unswizzled images)
  }
  for (int i = threadIdx.x; i < grow * KP / 16; i += 256) {
    *(uint4*)(gimg + Pmax * grow + 16 * i) = uint4{0u, 0u, 0u, 0u};
    if constexpr (DMA) *(uint4*)(gimg + SB + Pmax * grow + 16 * i) = uint4{0u, 0u, 0u, 0u};
  }
  // DMA: stage (gs, xs: gq g chunks, xq x chunks) into buffer `buf`; wave w issues the 64-chunk groups
  // w, w + 4, ... of each image (lanes past its end masked off)
  auto dma_stage = [&](int buf, const char* gs, const char* xs, int gq_, int xq_) {
    char* gb = lds + buf * SB;
    char* xb = gb + (Pmax + KP) * grow;
    for (int k0 = wave * 64; k0 < gq_; k0 += 256) {
      const int k = k0 + lane;
      if (k < gq_) {
        const int row = k / (grow / 16), c = k % (grow / 16);
        const int cs = N == 64 ? c ^ (swz128(row) >> 4) : c;
        __builtin_amdgcn_global_load_lds((const void*)(gs + (size_t)row * grow + 16 * cs), (__attribute__((address_space(3))) void*)(gb + 16 * k0), 16, 0, 0);
      }
    }
    for (int k0 = wave * 64; k0 < xq_; k0 += 256) {
      const int k = k0 + lane;
      if (k < xq_) {
        const int row = k / (xrowb / 16), c = k % (xrowb / 16);
        const int cs = C == 64 ? c ^ (swz128(row) >> 4) : c;
        __builtin_amdgcn_global_load_lds((const void*)(xs + (size_t)row * xrowb + 16 * cs), (__attribute__((address_space(3))) void*)(xb + 16 * k0), 16, 0, 0);
      }
    }
  };

  typename M::acc_t acc[TW][AN][AC];
#pragma unroll
  for (int t = 0; t < TW; ++t)
#pragma unroll
    for (int nb = 0; nb < AN; ++nb)
#pragma unroll
      for (int cb = 0; cb < AC; ++cb) acc[t][nb][cb] = typename M::acc_t{};

  const int stages_per_sample = (Ho + R - 1) / R;
  const int nstages = (b1 - b0) * stages_per_sample;
  // lane-constant parts of the tr-read addresses
  const int acol0 = (16 * gh + 4 * pp) * 2;  // + nb * MS * 2 bytes
  uint4 buf0, buf1, buf2, buf3, buf4, buf5, buf6, buf7, buf8, buf9, buf10, buf11;  // kWgradPieces
  int gq = 0, xq = 0;
  if (nstages > 0) {
    const int y0 = 0, nr = min(R, Ho);
    gq = nr * Wo * grow / 16;
    xq = min(nr + TKY - 1, H - kyA) * W * xrowb / 16;
    const char* gs = (const char*)g + ((size_t)b0 * Ho + y0) * Wo * grow;
    const char* xs = (const char*)x + ((size_t)b0 * H + y0 + kyA) * W * xrowb;
    if constexpr (DMA) {
      dma_stage(0, gs, xs, gq, xq);
    } else {
      FFMP_WGRAD_LOAD(gs, xs)
    }
  }
  for (int st = 0; st < nstages; ++st) {
    if constexpr (DMA) {
      // stage st landed (the barrier's vmcnt(0)), and every wave is done with buffer (st + 1) & 1
      __syncthreads();
      gimg = lds + (st & 1) * SB;
      ximg = gimg + (Pmax + KP) * grow;
    } else {
      __syncthreads();  // the previous stage's reads are done
      FFMP_WGRAD_STORE()
      __syncthreads();
    }
    const int nr = min(R, Ho - (st % stages_per_sample) * R);
    if (st + 1 < nstages) {  // the next stage, in flight while this one is consumed
      const int b = b0 + (st + 1) / stages_per_sample, y0 = ((st + 1) % stages_per_sample) * R;
      const int nr1 = min(R, Ho - y0);
      gq = nr1 * Wo * grow / 16;
      xq = min(nr1 + TKY - 1, H - y0 - kyA) * W * xrowb / 16;
      const char* gs = (const char*)g + ((size_t)b * Ho + y0) * Wo * grow;
      const char* xs = (const char*)x + ((size_t)b * H + y0 + kyA) * W * xrowb;
      if constexpr (DMA) {
        dma_stage((st + 1) & 1, gs, xs, gq, xq);
      } else {
        FFMP_WGRAD_LOAD(gs, xs)
      }
    }
    const int Ps = nr * Wo;
    // this lane's two k rows per k-step (u = 0, 1): position p = k0 + 8 fk + 4u + q, as (stage
    // row, column), advanced by KP per k-step without branches on data (Wo >= 8: host check); xo = the
    // byte offset of its x image row (pr W + pc) xrowb, advanced with it (no multiply per k-step)
    int pr[2], pc[2], xo[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int p = 8 * fk + 4 * u + q;
      pr[u] = p / Wo;
      pc[u] = p - pr[u] * Wo;
      xo[u] = (pr[u] * W + pc[u]) * xrowb;
    }
    const int xwrap = (W - Wo) * xrowb;  // x bytes skipped when a position row wraps
    // each operand fragment = two transposing reads (k rows 8 fk + 4u .. +4), joined as whole
    // vectors (element-wise assembly of the 4 x 16-bit results miscompiles: ROCm 7.2)
    auto fetch = [&](int k0, s16x4 (&ar)[AN][2], s16x4 (&br)[TW][AC][2]) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int p = k0 + 8 * fk + 4 * u + q;
        const bool in = p < Ps;
        const int grw = in ? p : Pmax + (p & (KP - 1));  // past the stage end: a zero row
#pragma unroll
        for (int nb = 0; nb < AN; ++nb) {
          const int col = acol0 + nb * MS * 2;
          const int off = N == 64 ? ((col & ~15) ^ swz128(grw)) | (col & 15) : col;
          ar[nb][u] = tr_read(gimg + grw * grow + off);
        }
        const int base = in ? pr[u] * W + pc[u] : 0;  // (C = 64: xo in C = 32's form below)
        if constexpr (C == 64) {  // 128-byte rows: the chunk swizzle depends on each read's row
#pragma unroll
          for (int t = 0; t < TW; ++t) {
            const int xrw = base + dky[t] * W + dkx[t];
#pragma unroll
            for (int cb = 0; cb < AC; ++cb) {
              const int col = acol0 + cb * MS * 2;
              br[t][cb][u] = tr_read(ximg + xrw * xrowb + (((col & ~15) ^ swz128(xrw)) | (col & 15)));
            }
          }
        } else {  // one lane address per k row, plus a scalar tap offset and a constant column offset
          const char* xl = ximg + (in ? xo[u] : 0) + acol0;
#pragma unroll
          for (int t = 0; t < TW; ++t)
#pragma unroll
            for (int cb = 0; cb < AC; ++cb) br[t][cb][u] = tr_read(xl + toff[t] + cb * MS * 2);
        }
        int c = pc[u] + KP, rr = pr[u], xr = xo[u] + KP * xrowb;
        if (c >= Wo) c -= Wo, ++rr, xr += xwrap;
        if (Wo < KP) {  // rows shorter than a k-step: up to KP / 8 wraps in all (Wo >= 8: host check)
#pragma unroll
          for (int wrap = 1; wrap < KP / 8; ++wrap)
            if (c >= Wo) c -= Wo, ++rr, xr += xwrap;
        }
        pc[u] = c;
        pr[u] = rr;
        xo[u] = xr;
      }
    };
    auto mma = [&](const s16x4 (&ar)[AN][2], const s16x4 (&br)[TW][AC][2]) {
      bf16x8 a[AN], bb[TW][AC];
#pragma unroll
      for (int nb = 0; nb < AN; ++nb)
        a[nb] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(ar[nb][0], ar[nb][1], 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
      for (int t = 0; t < TW; ++t)
#pragma unroll
        for (int cb = 0; cb < AC; ++cb)
          bb[t][cb] = __builtin_bit_cast(bf16x8,
                                         __builtin_shufflevector(br[t][cb][0], br[t][cb][1], 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
      for (int t = 0; t < TW; ++t)
#pragma unroll
        for (int nb = 0; nb < AN; ++nb)
#pragma unroll
          for (int cb = 0; cb < AC; ++cb) acc[t][nb][cb] = M::mma(a[nb], bb[t][cb], acc[t][nb][cb]);
    };
    constexpr bool kPrefetch = PF || (FFMP_WGRAD_PREFETCH < 0 ? TW * AN * AC * (MS / 16) * (MS / 16) >= 64
                                                             : FFMP_WGRAD_PREFETCH != 0);
    if constexpr (kPrefetch) {
      // the next k-step's fragments are read while this one's MFMAs run (two register sets, the loop
      // unrolled by two so they swap roles without copies)
      s16x4 arA[AN][2], brA[TW][AC][2], arB[AN][2], brB[TW][AC][2];
      fetch(0, arA, brA);
      for (int k0 = 0; k0 < Ps; k0 += 2 * KP) {
        fetch(k0 + KP, arB, brB);
        mma(arA, brA);
        if (k0 + KP >= Ps) break;
        fetch(k0 + 2 * KP, arA, brA);
        mma(arB, brB);
      }
    } else {
      for (int k0 = 0; k0 < Ps; k0 += KP) {
        s16x4 ar[AN][2], br[TW][AC][2];
        fetch(k0, ar, br);
        mma(ar, br);
      }
    }
  }

  // partial sums: part[chunk][tap][n][c]; C/D row = n (nb MS + Mfma<MS>::row(i, fk)), column = c (fr)
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    const int k = wave * TW + t;
    float* dst = part + ((size_t)blockIdx.y * KH * KW + (kyA + k / TKX) * KW + kxA + k % TKX) * N * C;
#pragma unroll
    for (int nb = 0; nb < AN; ++nb)
#pragma unroll
      for (int cb = 0; cb < AC; ++cb)
#pragma unroll
        for (int i = 0; i < M::NACC; ++i) {
          const int n = nb * MS + M::row(i, fk);
          dst[n * C + cb * MS + fr] = acc[t][nb][cb][i];
        }
  }
}

template <int C, int N, int TW>
int launch_wgrad(const void* g, const void* x, float* part, int B, int H, int W, int KH, int KW, int dx, int chunks,
                 hipStream_t s) {
  const int Ho = H - KH + 1, Wo = W - (KW - 1) * dx;
  constexpr int TG = 4 * TW;
  const int TKX = std::min(KW, TG), TKY = TG / TKX;
  if (KW % TKX || KH % TKY) return fail(FFMP_E_ARG, "ffmp_conv2d_wgrad: kernel %d x %d does not tile by %d taps", KH, KW, TG);
  // stage rows R: the most rows whose g + x images fit 48 KiB of LDS and 12 register pieces
  // MFMA shape: 16x16x32 by default except for the 32 -> 64 layer (conv2: 1.35 vs 1.66 ms on 16x16x32, and
  // its LDS-DMA stages below are built for 32x32x16); the other layers' weight gradients ran faster on it
  // (conv1 folded 0.415 -> 0.352 ms, conv3 0.186 -> 0.162, conv4 0.118 -> 0.111 at B = 256;
  // profiles/r06j_conv_ab_wgrad_ms16.txt)
  const int ms = ffmp_detail::mfma_for(C == 32 && N == 64 ? 32 : 16) == 16 ? 16 : 32, kp = ms == 16 ? 32 : 16;  // + kp zero g rows
  // LDS-DMA staging into two stage buffers with the k-step prefetch (FFMP_TUNE_CONV_WGDMA), the 32x32x16
  // shape, stages of up to 8 rows in 2 x 80 KiB.  Default: where the kernel holds one workgroup per CU
  // anyway (more than 8 accumulator blocks per wave: conv2's 32 -> 64, 1.70 -> 1.47 ms at B = 256,
  // 6.69 -> 5.75 ms at 1,024); the 2 x 80 KiB would cost the smaller ones their second and third
  // workgroup per CU (conv3's 64 -> 64: 0.180 -> 0.242 ms; profiles/r06e_conv_ab_wgdma.txt)
  int wgdma = 0;
  if (ms == 32) {
    const int knob = ffmp_detail::g_conv_wgdma;
    wgdma = knob == 3 ? 0 : knob == 4 ? 2 : knob != 0 ? knob : (TW * (N / 32) * (C / 32) > 8 ? 2 : 0);
  }
  // two stage buffers per workgroup: 2 x 80 KiB where the kernel holds one workgroup per CU anyway,
  // 2 x 40 KiB (two workgroups per CU) otherwise
  const size_t stage_cap = TW * (N / 32) * (C / 32) > 8 ? 80 * 1024 : 40 * 1024;
  int R = std::min(Ho, 8);
  auto bytes = [&](int rr) { return (size_t)(rr * Wo + kp) * N * 2 + (size_t)(rr + TKY - 1) * W * C * 2; };
  auto pieces = [&](int rr) { return ((size_t)rr * Wo * N * 2 + (size_t)(rr + TKY - 1) * W * C * 2) / 16; };
  if (wgdma) {
    while (R > 1 && bytes(R) > stage_cap) --R;
    if (bytes(R) > stage_cap)
      return fail(FFMP_E_ARG, "ffmp_conv2d_wgrad: rows of %d x %d x %d do not fit one stage", W, C, N);
  } else {
    while (R > 1 && (bytes(R) > 48 * 1024 || pieces(R) > kWgradPieces * 256)) --R;
    if (bytes(R) > 64 * 1024 || pieces(R) > kWgradPieces * 256)
      return fail(FFMP_E_ARG, "ffmp_conv2d_wgrad: rows of %d x %d x %d do not fit one stage", W, C, N);
  }
  if (Wo < 8) return fail(FFMP_E_ARG, "ffmp_conv2d_wgrad: output rows of %d < 8 positions", Wo);
  const int per_chunk = (B + chunks - 1) / chunks;
  const dim3 grid((KH / TKY) * (KW / TKX), (B + per_chunk - 1) / per_chunk);
  if (t_conv_dry) return FFMP_OK;
  auto go = [&](auto MS_, auto PF_) {
    hipLaunchKernelGGL((conv_wgrad_kernel<C, N, TW, decltype(MS_)::value, decltype(PF_)::value>), grid, dim3(256),
                       bytes(R), s, (const __bf16*)g, (const __bf16*)x, part, B, H, W, KH, KW, dx, TKY, TKX, R,
                       per_chunk);
  };
  const bool pf = ffmp_detail::g_conv_wgpf != 0;
  if (wgdma) {
    if (wgdma == 2)
      hipLaunchKernelGGL((conv_wgrad_kernel<C, N, TW, 32, true, true>), grid, dim3(256), 2 * bytes(R), s,
                         (const __bf16*)g, (const __bf16*)x, part, B, H, W, KH, KW, dx, TKY, TKX, R, per_chunk);
    else
      hipLaunchKernelGGL((conv_wgrad_kernel<C, N, TW, 32, false, true>), grid, dim3(256), 2 * bytes(R), s,
                         (const __bf16*)g, (const __bf16*)x, part, B, H, W, KH, KW, dx, TKY, TKX, R, per_chunk);
  } else if (ms == 16) {
    if (pf) go(std::integral_constant<int, 16>{}, std::true_type{});
    else go(std::integral_constant<int, 16>{}, std::false_type{});
  } else {
    if (pf) go(std::integral_constant<int, 32>{}, std::true_type{});
    else go(std::integral_constant<int, 32>{}, std::false_type{});
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(FFMP_E_HIP, "ffmp_conv2d_wgrad launch: %s", hipGetErrorString(e));
  return FFMP_OK;
}

// ------------------------------------------------------------------ data gradient, samples as M
// dX[b][Y][X][n] = sum_{ky, kx, c} g[b][Y + ky - (KH-1)][X + kx - (KW-1)][c] * w'[ky][kx][n][c]: the full
// convolution of the output gradient g (NHWC [B][Hy][Wy][C]) with the flipped, transposed kernel
// (conv_mfma.pack_weight_dgrad).  As an implicit GEMM over output positions (conv_fwd_kernel with
// pad = k - 1) a 32-position block spans a whole ramp of valid kernel columns and issues ~1.8x its
// useful products at conv2's shape (a 69-wide output row, a 38-wide gradient, 32 kernel columns).
// Here the GEMM's M is 32 SAMPLES of one output position: every row of an MFMA block has the same
// valid taps, so a wave issues exactly the useful products — a tap (ky, kx) is skipped for the
// whole block when its gradient cell falls outside the image (wave-uniform tests, no zero products).
//   A = g[32 samples][16 channels of one gradient cell] (LDS), B = w'[tap][16 channels][32 n] (L1),
//   D[sample][n] accumulates per output position, fp32.
// A workgroup = NW waves owns one output row Y of one group of 32 samples; wave w owns the NW-strided
// positions X = w + NW * i (i < PW), so all waves see the same share of each kernel column's valid
// window (the parallelogram {(X, kx): 0 <= X + kx - (KW-1) < Wy}) and reach the per-phase barrier
// together.  Phase = (ky, KQ k-steps of channels): the gradient row u = Y + ky - (KH-1), those
// channels, every column, 32 samples — KQ KiB per column, laid out [v][k-step][h][sample][8] so a
// fragment read is 1 KiB of consecutive bytes (ds_read_b128, conflict-free) — sits in one of two
// LDS buffers; the next phase's row is loaded piece by piece (1 KiB per wave-instruction, a piece
// per kernel column) into the other buffer during the sweep and published by the phase's barrier.
// Rows are dealt heaviest first (the middle output rows meet all KH kernel rows, the border rows
// one), so the last workgroups to start are the short ones.
// Measured and not kept (conv2's data gradient at B = 256, 1.59-1.62 ms with this code;
// profiles/r05d_dgrad_ahead.txt, r05f_dgrad_variants.txt): A fragments read one valid position ahead
// behind the guards (1.83 ms); B fragments and next-phase pieces over two register sets that swap
// roles (1.63-1.64); one k-step per phase (2.26; with every valid position's A requested first 2.73);
// 4 waves x 18 positions at one wave per SIMD (2.64); valid positions two at a time (490 spilled VGPRs).
constexpr int kDgradNW = 8, kDgradPW = 9, kDgradKQ = 2;  // 72 output columns per row, 2 waves/SIMD

template <int C, int N, int NW, int PW, int KQ, int MS = 32>
__global__ __launch_bounds__(NW * 64, 1) void conv_dgrad_bm_kernel(const __bf16* __restrict__ g,
                                                                 const __bf16* __restrict__ w,
                                                                 void* __restrict__ y, int B, int Hy, int Wy,
                                                                 int KH, int KW, int flags) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  using M = Mfma<MS>;
  constexpr int NQ = C / (16 * KQ);  // phases per kernel row
  // MFMA blocks per position: samples (32 = AM x MS) x output channels (N = AN x MS); k-steps of
  // M::KS channels per phase (MS = 16: one of 32 = the phase's KQ = 2 chunks of 16)
  constexpr int AM = 32 / MS, AN = N / MS, KSTEPS = KQ * 16 / M::KS;
  static_assert(KSTEPS >= 1 && KQ * 16 % M::KS == 0, "a phase holds whole k-steps");
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;          // the staging lanes: sample r, channel half h
  const int fr = lane & (MS - 1), fk = lane / MS;  // the operand lanes: row, k-chunk of 8 channels
  const int G = (B + 31) / 32;
  const int rank = blockIdx.x / G, grp = blockIdx.x % G;
  const int padY = KH - 1, padX = KW - 1;
  const int Hx = Hy + padY, Wx = Wy + padX;
  const int Yc = (Hx - 1) / 2;  // rank 0, 1, 2, ... -> Yc, Yc + 1, Yc - 1, ...: most kernel rows first
  const int Y = (rank & 1) ? Yc + (rank + 1) / 2 : Yc - rank / 2;
  const int b0 = grp * 32;
  const int ky_lo = max(0, padY - Y), ky_hi = min(KH - 1, padY + Hy - 1 - Y);
  const int nph = (ky_hi - ky_lo + 1) * NQ;
  const int colb = KQ * 1024;  // bytes of one gradient column in a buffer
  const int bufb = Wy * colb;
  const int npieces = Wy * KQ;
  // this lane's sample (ragged last group: the last sample again; those rows are never stored)
  const char* gs = (const char*)g + (size_t)min(b0 + r, B - 1) * Hy * Wy * C * 2;
  // piece p of phase (u, q): column v = p / KQ, k-step s = p % KQ; lane (r, h) brings channels
  // (q KQ + s) 16 + 8h .. +8 of its sample
  auto piece = [&](int u, int q, int p) -> uint4 {
    const int v = p / KQ, s = p - (p / KQ) * KQ;
    return *(const uint4*)(gs + ((size_t)u * Wy + v) * C * 2 + ((q * KQ + s) * 16 + 8 * h) * 2);
  };
  auto piece_lds = [&](int buf, int p) -> uint4* { return (uint4*)(lds + buf * bufb + p * 1024 + lane * 16); };
  // the A fragment (samples mb MS + fr, channel chunk kc = 2 k-step-of-16 + half) inside a column:
  // chunk kc of sample b sits at (kc / 2) 1024 + (kc & 1) 512 + b 16
  auto a_off = [&](int s, int mb) -> int {
    const int kc = s * (M::KS / 8) + fk;
    return (kc >> 1) * 1024 + (kc & 1) * 512 + (mb * MS + fr) * 16;
  };

  {  // phase 0 into buffer 0
    const int u0 = Y + ky_lo - padY;
    for (int p = wave; p < npieces; p += NW) *piece_lds(0, p) = piece(u0, 0, p);
  }
  __syncthreads();

  typename M::acc_t acc[PW][AM][AN];
#pragma unroll
  for (int i = 0; i < PW; ++i)
#pragma unroll
    for (int mb = 0; mb < AM; ++mb)
#pragma unroll
      for (int nb = 0; nb < AN; ++nb) acc[i][mb][nb] = typename M::acc_t{};

  // B fragments of tap t, the phase's k-steps: w [KH][KW][C/8][N][8]: lane (fr, fk) of k-step ks reads
  // chunk (q KQ 16 + ks KS) / 8 + fk, n = nb MS + fr — MS x 16 bytes of consecutive memory per chunk
  auto load_b = [&](int t, int q, bf16x8 (&dst)[KSTEPS][AN]) {
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s)
#pragma unroll
      for (int nb = 0; nb < AN; ++nb)
        dst[s][nb] = *(const bf16x8*)(w + (((size_t)t * (C / 8) + (q * KQ * 16 + s * M::KS) / 8 + fk) * N + nb * MS + fr) * 8);
  };

  for (int ph = 0; ph < nph; ++ph) {
    const int ky = ky_lo + ph / NQ, q = ph % NQ, buf = ph & 1;
    const bool more = ph + 1 < nph;
    const int u1 = Y + ky_lo + (ph + 1) / NQ - padY, q1 = (ph + 1) % NQ;
    bf16x8 bcur[KSTEPS][AN];
    load_b(ky * KW, q, bcur);
    uint4 pc = uint4{0u, 0u, 0u, 0u};
    int pprev = -1;  // the piece held in pc, written one kernel column later
    for (int j = 0; j < KW; ++j) {
      bf16x8 bnx[KSTEPS][AN];
      load_b(ky * KW + min(j + 1, KW - 1), q, bnx);
      if (more) {
        if (pprev >= 0) *piece_lds(buf ^ 1, pprev) = pc;
        const int p = wave + NW * j;
        pprev = p < npieces ? p : -1;
        if (pprev >= 0) pc = piece(u1, q1, p);
      }
      // this wave's positions whose gradient column v = X + j - padX lies in [0, Wy): i in [ilo, ihi]
      const int t0 = padX - j - wave;
      const int ilo = t0 <= 0 ? 0 : (t0 + NW - 1) / NW;
      const int t1 = min(padX + Wy - 1 - j, Wx - 1) - wave;
      const int ihi = t1 < 0 ? -1 : min(PW - 1, t1 / NW);
      const char* abase = lds + buf * bufb + (wave + j - padX) * colb;
#pragma unroll
      for (int i = 0; i < PW; ++i) {
        if (i >= ilo && i <= ihi) {
          bf16x8 a[KSTEPS][AM];
#pragma unroll
          for (int s = 0; s < KSTEPS; ++s)
#pragma unroll
            for (int mb = 0; mb < AM; ++mb) a[s][mb] = *(const bf16x8*)(abase + NW * i * colb + a_off(s, mb));
#pragma unroll
          for (int s = 0; s < KSTEPS; ++s)
#pragma unroll
            for (int mb = 0; mb < AM; ++mb)
#pragma unroll
              for (int nb = 0; nb < AN; ++nb) acc[i][mb][nb] = M::mma(a[s][mb], bcur[s][nb], acc[i][mb][nb]);
        }
      }
#pragma unroll
      for (int s = 0; s < KSTEPS; ++s)
#pragma unroll
        for (int nb = 0; nb < AN; ++nb) bcur[s][nb] = bnx[s][nb];
    }
    if (more) {
      if (pprev >= 0) *piece_lds(buf ^ 1, pprev) = pc;
      for (int p = wave + NW * KW; p < npieces; p += NW) *piece_lds(buf ^ 1, p) = piece(u1, q1, p);  // KW < pieces / NW
    }
    __syncthreads();
  }

  // epilogue: D row = sample mb MS + Mfma<MS>::row(e, fk), column = n (fr)
  const bool out_bf16 = flags & FFMP_CONV_OUT_BF16;
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int X = wave + NW * i;
    if (X >= Wx) continue;
#pragma unroll
    for (int mb = 0; mb < AM; ++mb)
#pragma unroll
      for (int nb = 0; nb < AN; ++nb)
#pragma unroll
        for (int e = 0; e < M::NACC; ++e) {
          const int b = b0 + mb * MS + M::row(e, fk);
          if (b >= B) continue;
          const size_t o = (((size_t)b * Hx + Y) * Wx + X) * N + nb * MS + fr;
          if (out_bf16)
            ((__bf16*)y)[o] = (__bf16)acc[i][mb][nb][e];
          else
            ((float*)y)[o] = acc[i][mb][nb][e];
        }
  }
}

template <int C, int N>
int launch_dgrad_bm(const void* g, const void* w, void* y, int B, int Hy, int Wy, int KH, int KW, int flags,
                    hipStream_t s) {
  constexpr int NW = kDgradNW, PW = kDgradPW, KQ = kDgradKQ;
  const int Hx = Hy + KH - 1, Wx = Wy + KW - 1;
  const size_t lds = (size_t)2 * Wy * KQ * 1024;
  if (Wx > NW * PW) return fail(FFMP_E_ARG, "ffmp_conv2d_dgrad: output rows of %d > %d positions", Wx, NW * PW);
  if (lds > 160 * 1024)
    return fail(FFMP_E_ARG, "ffmp_conv2d_dgrad: two gradient rows of %d cells (%zu bytes) exceed the 160 KiB LDS", Wy, lds);
  const long blocks = (long)Hx * ((B + 31) / 32);
  if (blocks > 0x7fffffffL) return fail(FFMP_E_ARG, "ffmp_conv2d_dgrad: grid too large");
  if (t_conv_dry) return FFMP_OK;
  if (ffmp_detail::mfma_for(32) == 16)
    hipLaunchKernelGGL((conv_dgrad_bm_kernel<C, N, NW, PW, KQ, 16>), dim3((unsigned)blocks), dim3(NW * 64), lds, s,
                       (const __bf16*)g, (const __bf16*)w, y, B, Hy, Wy, KH, KW, flags);
  else
    hipLaunchKernelGGL((conv_dgrad_bm_kernel<C, N, NW, PW, KQ, 32>), dim3((unsigned)blocks), dim3(NW * 64), lds, s,
                       (const __bf16*)g, (const __bf16*)w, y, B, Hy, Wy, KH, KW, flags);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(FFMP_E_HIP, "ffmp_conv2d_dgrad launch: %s", hipGetErrorString(e));
  return FFMP_OK;
}

}  // namespace

extern "C" {

int ffmp_conv2d_fwd_bf16(const void* x, const void* w, const float* bias, void* y, int32_t batch, int32_t h,
                         int32_t wd, int32_t c, int32_t kh, int32_t kw, int32_t n, int32_t pad, int32_t dx,
                         int32_t flags, void* stream) {
  if (!x || !w || !y) return fail(FFMP_E_ARG, "ffmp_conv2d_fwd_bf16: NULL tensor");
  if (batch <= 0 || batch > 65535 || kh <= 0 || kw <= 0 || pad < 0 || pad >= kh || pad >= kw || dx < 1 ||
      h + 2 * pad < kh || wd + 2 * pad < (kw - 1) * dx + 1)
    return fail(FFMP_E_ARG, "ffmp_conv2d_fwd_bf16: bad shape (batch %d, %d x %d input, %d x %d kernel, pad %d, dx %d)",
                batch, h, wd, kh, kw, pad, dx);
  if (((uintptr_t)x | (uintptr_t)w) & 15) return fail(FFMP_E_ARG, "ffmp_conv2d_fwd_bf16: x and w must be 16-byte aligned");
  if (flags & ~(FFMP_CONV_RELU | FFMP_CONV_OUT_BF16 | FFMP_CONV_W_FRAG | FFMP_CONV_X_FOLD))
    return fail(FFMP_E_ARG, "ffmp_conv2d_fwd_bf16: unknown flags 0x%x", flags);
  if ((flags & FFMP_CONV_X_FOLD) && (dx < 2 || c % dx || ((c / dx) * 2) % 4 || pad))
    return fail(FFMP_E_ARG, "ffmp_conv2d_fwd_bf16: FFMP_CONV_X_FOLD needs dx >= 2 dividing c into an even channel count "
                "and pad 0 (got c %d, dx %d, pad %d)", c, dx, pad);
  hipStream_t s = (hipStream_t)stream;
  if (pad > 0) {  // data gradients of the 32/64-channel convolutions (c = their output channels)
    if (c == 64 && n == 32) return launch_fwd<64, 1, true>(x, w, bias, y, batch, h, wd, kh, kw, pad, dx, flags, s);
    if (c == 64 && n == 64) return launch_fwd<64, 2, true>(x, w, bias, y, batch, h, wd, kh, kw, pad, dx, flags, s);
    if (c == 32 && n == 64) return launch_fwd<32, 2, true>(x, w, bias, y, batch, h, wd, kh, kw, pad, dx, flags, s);
    if (c == 32 && n == 32) return launch_fwd<32, 1, true>(x, w, bias, y, batch, h, wd, kh, kw, pad, dx, flags, s);
  }
  if (c == 32 && n == 64) return launch_fwd<32, 2, false>(x, w, bias, y, batch, h, wd, kh, kw, 0, dx, flags, s);
  if (c == 64 && n == 64) return launch_fwd<64, 2, false>(x, w, bias, y, batch, h, wd, kh, kw, 0, dx, flags, s);
  if (c == 64 && n == 32) return launch_fwd<64, 1, false>(x, w, bias, y, batch, h, wd, kh, kw, 0, dx, flags, s);
  if (c == 32 && n == 32) return launch_fwd<32, 1, false>(x, w, bias, y, batch, h, wd, kh, kw, 0, dx, flags, s);
  return fail(FFMP_E_ARG, "ffmp_conv2d_fwd_bf16: channels in/out must be 32 or 64 (got %d / %d)", c, n);
}

int ffmp_conv2d_wgrad_bf16(const void* g, const void* x, float* part, int32_t batch, int32_t h, int32_t wd, int32_t c,
                           int32_t kh, int32_t kw, int32_t n, int32_t dx, int32_t chunks, void* stream) {
  if (!g || !x || !part) return fail(FFMP_E_ARG, "ffmp_conv2d_wgrad_bf16: NULL tensor");
  if (batch <= 0 || batch > 65535 || kh <= 0 || kw <= 0 || dx < 1 || h < kh || wd < (kw - 1) * dx + 1 || chunks < 1)
    return fail(FFMP_E_ARG, "ffmp_conv2d_wgrad_bf16: bad shape (batch %d, %d x %d input, %d x %d kernel, dx %d, %d chunks)",
                batch, h, wd, kh, kw, dx, chunks);
  if (((uintptr_t)g | (uintptr_t)x) & 15) return fail(FFMP_E_ARG, "ffmp_conv2d_wgrad_bf16: g and x must be 16-byte aligned");
  hipStream_t s = (hipStream_t)stream;
  if (c == 32 && n == 64) {  // FFMP_TUNE_CONV_WGDMA 4: 4 taps per wave, LDS-DMA stages, two workgroups per CU
    if (ffmp_detail::g_conv_wgdma == 4) return launch_wgrad<32, 64, 4>(g, x, part, batch, h, wd, kh, kw, dx, chunks, s);
    return launch_wgrad<32, 64, FFMP_WGRAD_TW_3264>(g, x, part, batch, h, wd, kh, kw, dx, chunks, s);
  }
  if (c == 64 && n == 64) return launch_wgrad<64, 64, 2>(g, x, part, batch, h, wd, kh, kw, dx, chunks, s);
  if (c == 32 && n == 32) return launch_wgrad<32, 32, 2>(g, x, part, batch, h, wd, kh, kw, dx, chunks, s);
  if (c == 64 && n == 32) return launch_wgrad<64, 32, 4>(g, x, part, batch, h, wd, kh, kw, dx, chunks, s);
  return fail(FFMP_E_ARG, "ffmp_conv2d_wgrad_bf16: channels in/out must be 32 or 64 (got %d / %d)", c, n);
}

int ffmp_conv2d_dgrad_bf16(const void* g, const void* w, void* dx, int32_t batch, int32_t hy, int32_t wy, int32_t c,
                           int32_t kh, int32_t kw, int32_t n, int32_t flags, void* stream) {
  if (!g || !w || !dx) return fail(FFMP_E_ARG, "ffmp_conv2d_dgrad_bf16: NULL tensor");
  if (batch <= 0 || hy <= 0 || wy <= 0 || kh <= 0 || kw <= 0)
    return fail(FFMP_E_ARG, "ffmp_conv2d_dgrad_bf16: bad shape (batch %d, %d x %d gradient, %d x %d kernel)", batch, hy,
                wy, kh, kw);
  if (((uintptr_t)g | (uintptr_t)w) & 15) return fail(FFMP_E_ARG, "ffmp_conv2d_dgrad_bf16: g and w must be 16-byte aligned");
  hipStream_t s = (hipStream_t)stream;
  if (c == 64 && n == 32) return launch_dgrad_bm<64, 32>(g, w, dx, batch, hy, wy, kh, kw, flags, s);
  if (c == 32 && n == 32) return launch_dgrad_bm<32, 32>(g, w, dx, batch, hy, wy, kh, kw, flags, s);
  return fail(FFMP_E_ARG, "ffmp_conv2d_dgrad_bf16: gradient channels 32 or 64 and 32 output channels (got %d / %d)", c, n);
}

int ffmp_conv2d_check(int32_t kind, int32_t batch, int32_t h, int32_t wd, int32_t c, int32_t kh, int32_t kw,
                      int32_t n, int32_t pad, int32_t dx) {
  // aligned stand-in pointers: nothing is read or launched in a dry run
  void* const p = reinterpret_cast<void*>(static_cast<uintptr_t>(256));
  t_conv_dry = true;
  const int rc = kind == 0 ? ffmp_conv2d_fwd_bf16(p, p, nullptr, p, batch, h, wd, c, kh, kw, n, pad, dx, 0, nullptr)
               : kind == 1 ? ffmp_conv2d_wgrad_bf16(p, p, static_cast<float*>(p), batch, h, wd, c, kh, kw, n, dx, 1, nullptr)
               : kind == 2 ? ffmp_conv2d_dgrad_bf16(p, p, p, batch, h, wd, c, kh, kw, n, 0, nullptr)
                           : fail(FFMP_E_ARG, "ffmp_conv2d_check: kind must be 0 (forward / data gradient), 1 (weight gradient) or 2 (data gradient, samples as M)");
  t_conv_dry = false;
  return rc;
}

}  // extern "C"
