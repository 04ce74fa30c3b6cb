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

#include "ffmp.h"

namespace ffmp_detail {
int fail(int code, const char* fmt, ...);  // ffmp_kernels.hip (sets ffmp_last_error())
}
using ffmp_detail::fail;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kWaves = 4;

template <int C>
__device__ __forceinline__ void load_row_regs(const char* __restrict__ src, int chunks, uint4 (&buf)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = threadIdx.x + 256 * i;
    if (q < chunks) buf[i] = src ? *(const uint4*)(src + 16 * (size_t)q) : uint4{0u, 0u, 0u, 0u};
  }
}

__device__ __forceinline__ void store_row_lds(char* dst, int chunks, const uint4 (&buf)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = threadIdx.x + 256 * i;
    if (q < chunks) *(uint4*)(dst + 16 * q) = buf[i];
  }
}

// Implicit zero padding of `pad` cells on every side: logical input rows/columns [pad, pad + H/W)
// hold the tensor, the rest are zero.  A ring slot is Wp = W + 2 pad cells wide; its pad columns
// are zeroed once, a row load writes the W real cells (or zeros for a row outside the tensor).
// The ky loop runs only over kernel rows for which some row of the tile touches the tensor, and a
// wave skips the MFMAs of kernel rows its own positions never see (the data gradient's k - 1 zero
// border: ~12 % of its work).  Kernel column kx reads input column xp + kx * dx (dx > 1: the
// x-dilated form a 1- or 2-channel convolution takes after its kernel columns are folded into
// channels, conv_mfma.fold_input).
template <int C, int NB, int MBW>
__global__ __launch_bounds__(256, 2) void conv_fwd_kernel(const __bf16* __restrict__ x, const __bf16* __restrict__ w,
                                                          const float* __restrict__ bias, void* __restrict__ y, int H,
                                                          int W, int KH, int KW, int pad, int dx, int RING, int flags) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  constexpr int N = NB * 32;
  constexpr int PT = kWaves * MBW * 32;
  const int Wp = W + 2 * pad;
  const int Ho = H + 2 * pad - KH + 1, Wo = Wp - (KW - 1) * dx;
  const int b = blockIdx.y;
  const int P = Ho * Wo;
  const int p0 = blockIdx.x * PT;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  const int rowbytes = W * C * 2;      // one tensor row
  const int slotbytes = Wp * C * 2;    // one ring slot
  const int chunks = rowbytes / 16;    // <= 4 * 256 (host check)
  const int yf = p0 / Wo;
  const int yl = min(P - 1, p0 + PT - 1) / Wo;
  const char* xb = (const char*)x + (size_t)b * H * rowbytes;
  // kernel rows whose input rows [yf + ky, yl + ky] meet the tensor rows [pad, pad + H) ...
  const int ky_lo = max(0, pad - yl), ky_hi = min(KH - 1, pad + H - 1 - yf);
  // ... and this wave's share of them (its positions' rows)
  const int pw0 = p0 + wave * MBW * 32;
  const int wyf = min(pw0, P - 1) / Wo, wyl = min(P - 1, pw0 + MBW * 32 - 1) / Wo;
  const int wk_lo = pw0 < P ? max(ky_lo, pad - wyl) : KH, wk_hi = min(ky_hi, pad + H - 1 - wyf);

  // this lane's output positions (clamped into the image; out-of-range ones are not stored)
  int ypos[MBW], xoff[MBW];
#pragma unroll
  for (int mb = 0; mb < MBW; ++mb) {
    const int m = min(p0 + (wave * MBW + mb) * 32 + r, P - 1);
    ypos[mb] = m / Wo;
    xoff[mb] = (m - ypos[mb] * Wo) * C * 2 + h * 16;
  }

  if (pad > 0) {  // the pad columns of every slot, once
    const int pchunks = pad * C * 2 / 16;
    for (int q = threadIdx.x; q < RING * 2 * pchunks; q += 256) {
      const int slot = q / (2 * pchunks), k = q % (2 * pchunks);
      const int off = k < pchunks ? 16 * k : (pad + W) * C * 2 + 16 * (k - pchunks);
      *(uint4*)(lds + slot * slotbytes + off) = uint4{0u, 0u, 0u, 0u};
    }
  }
  auto row_src = [&](int yr) -> const char* {  // logical row -> tensor row, or nullptr (zeros)
    const int real = yr - pad;
    return (real >= 0 && real < H) ? xb + (size_t)real * rowbytes : nullptr;
  };
  // ring rows for the first kernel row
  for (int row = yf + ky_lo; row <= yl + ky_lo; ++row) {
    uint4 buf[4];
    load_row_regs<C>(row_src(row), chunks, buf);
    store_row_lds(lds + (row % RING) * slotbytes + pad * C * 2, chunks, buf);
  }
  __syncthreads();

  f32x16 acc[MBW][NB];
#pragma unroll
  for (int mb = 0; mb < MBW; ++mb)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) acc[mb][nb] = f32x16{};

  // B fragments of the wave's first tap (wk_lo, 0); from then on loaded one tap ahead (the active
  // kernel rows [wk_lo, wk_hi] are consecutive)
  bf16x8 bcur[NB][C / 16];
  {
    const int t0 = min(wk_lo, KH - 1) * KW;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int s = 0; s < C / 16; ++s)
        bcur[nb][s] = *(const bf16x8*)(w + ((size_t)(t0 * N + nb * 32 + r) * C + s * 16 + h * 8));
  }

  for (int ky = ky_lo; ky <= ky_hi; ++ky) {
    uint4 nrow[4];
    const bool more = ky < ky_hi;
    if (more) load_row_regs<C>(row_src(yl + ky + 1), chunks, nrow);
    if (ky >= wk_lo && ky <= wk_hi) {
      int aoff[MBW];
#pragma unroll
      for (int mb = 0; mb < MBW; ++mb) aoff[mb] = ((ypos[mb] + ky) % RING) * slotbytes + xoff[mb];
      for (int kx = 0; kx < KW; ++kx) {
        // the next tap: (ky, kx + 1), else (ky + 1, 0) while the wave has rows left (the last
        // tap re-reads its own)
        const int tn = kx + 1 < KW ? ky * KW + kx + 1 : (ky < wk_hi ? (ky + 1) * KW : ky * KW + kx);
        bf16x8 bnext[NB][C / 16];
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
#pragma unroll
          for (int s = 0; s < C / 16; ++s)
            bnext[nb][s] = *(const bf16x8*)(w + ((size_t)(tn * N + nb * 32 + r) * C + s * 16 + h * 8));
        const int coff = kx * dx * C * 2;
#pragma unroll
        for (int s = 0; s < C / 16; ++s) {
          bf16x8 a[MBW];
#pragma unroll
          for (int mb = 0; mb < MBW; ++mb) a[mb] = *(const bf16x8*)(lds + aoff[mb] + coff + s * 32);
#pragma unroll
          for (int mb = 0; mb < MBW; ++mb)
#pragma unroll
            for (int nb = 0; nb < NB; ++nb)
              acc[mb][nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[mb], bcur[nb][s], acc[mb][nb], 0, 0, 0);
        }
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
#pragma unroll
          for (int s = 0; s < C / 16; ++s) bcur[nb][s] = bnext[nb][s];
      }
    }
    if (more) store_row_lds(lds + ((yl + ky + 1) % RING) * slotbytes + pad * C * 2, chunks, nrow);
    __syncthreads();
  }

  // epilogue: C/D of 32x32x16: column = lane & 31 (channel), row = (i & 3) + 8 (i >> 2) + 4 h
  const bool relu = flags & FFMP_CONV_RELU, out_bf16 = flags & FFMP_CONV_OUT_BF16;
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const int n = nb * 32 + r;
    const float bn = bias ? bias[n] : 0.f;
#pragma unroll
    for (int mb = 0; mb < MBW; ++mb) {
      const int mbase = p0 + (wave * MBW + mb) * 32;
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

// positions per workgroup: 512 (MBW 4), 256 or 128 — the fewest padded positions per image
// (ties to the larger tile); 256 at most when a 512-position ring would not leave room for two
// workgroups per CU (the data gradient's 100-cell padded rows)
int pick_mbw(int P, int Wo, size_t slotbytes) {
  int best = 4;
  long best_pad = -1;
  for (int mbw : {4, 2, 1}) {
    const int pt = kWaves * mbw * 32;
    const size_t ring = (size_t)((pt + Wo - 1) / Wo + 2) * slotbytes;
    if (ring > 80 * 1024 && mbw > 1) continue;
    const long padded = (long)((P + pt - 1) / pt) * pt;
    if (best_pad < 0 || padded < best_pad) best = mbw, best_pad = padded;
  }
  return best;
}

template <int C, int NB, int MBW>
int launch_fwd_mbw(const void* x, const void* w, const float* bias, void* y, int B, int H, int W, int KH, int KW,
                   int pad, int dx, int flags, hipStream_t s) {
  const int Ho = H + 2 * pad - KH + 1, Wo = W + 2 * pad - (KW - 1) * dx;
  constexpr int PT = kWaves * MBW * 32;
  const int span = (PT + Wo - 1) / Wo + 1;  // input rows a tile reads for one ky
  const int ring = span + 1;                // + the row loaded for the next ky
  const size_t lds = (size_t)ring * (W + 2 * pad) * C * 2;
  if (lds > 160 * 1024)
    return fail(FFMP_E_ARG, "ffmp_conv2d: a ring of %d input rows (%zu bytes) exceeds the 160 KiB LDS", ring, lds);
  if ((W * C * 2) / 16 > 4 * 256) return fail(FFMP_E_ARG, "ffmp_conv2d: input rows wider than 16 KiB");
  const dim3 grid((Ho * Wo + PT - 1) / PT, B);
  hipLaunchKernelGGL((conv_fwd_kernel<C, NB, MBW>), grid, dim3(256), lds, s, (const __bf16*)x, (const __bf16*)w, bias,
                     y, H, W, KH, KW, pad, dx, ring, flags);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(FFMP_E_HIP, "ffmp_conv2d launch: %s", hipGetErrorString(e));
  return FFMP_OK;
}

template <int C, int NB>
int launch_fwd(const void* x, const void* w, const float* bias, void* y, int B, int H, int W, int KH, int KW, int pad,
               int dx, int flags, hipStream_t s) {
  const int Ho = H + 2 * pad - KH + 1, Wo = W + 2 * pad - (KW - 1) * dx;
  switch (pick_mbw(Ho * Wo, Wo, (size_t)(W + 2 * pad) * C * 2)) {
    case 4: return launch_fwd_mbw<C, NB, 4>(x, w, bias, y, B, H, W, KH, KW, pad, dx, flags, s);
    case 2: return launch_fwd_mbw<C, NB, 2>(x, w, bias, y, B, H, W, KH, KW, pad, dx, flags, s);
    default: return launch_fwd_mbw<C, NB, 1>(x, w, bias, y, B, H, W, KH, KW, pad, dx, flags, s);
  }
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
  if ((pad * c * 2) % 16) return fail(FFMP_E_ARG, "ffmp_conv2d_fwd_bf16: pad * c must be a multiple of 8");
  hipStream_t s = (hipStream_t)stream;
  if (c == 32 && n == 64) return launch_fwd<32, 2>(x, w, bias, y, batch, h, wd, kh, kw, pad, dx, flags, s);
  if (c == 64 && n == 64) return launch_fwd<64, 2>(x, w, bias, y, batch, h, wd, kh, kw, pad, dx, flags, s);
  if (c == 64 && n == 32) return launch_fwd<64, 1>(x, w, bias, y, batch, h, wd, kh, kw, pad, dx, flags, s);
  if (c == 32 && n == 32) return launch_fwd<32, 1>(x, w, bias, y, batch, h, wd, kh, kw, pad, dx, flags, s);
  return fail(FFMP_E_ARG, "ffmp_conv2d_fwd_bf16: channels in/out must be 32 or 64 (got %d / %d)", c, n);
}

}  // extern "C"
