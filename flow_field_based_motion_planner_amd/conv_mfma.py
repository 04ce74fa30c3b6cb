"""The learner's dominant convolution on the MI355X matrix cores (include/ffmp.h
ffmp_conv2d_fwd_bf16).

The reference Network (/root/reference/src/train.py:231-303) is four stride-1 convolutions and
four linears; conv2 = nn.Conv2d(32, 64, kernel_size=32) (train.py:235) is ~80 % of its FLOPs
(6.06 GFLOP per sample forward at the reference's 100 x 100 map).  Under `Brain(amp=True)` it runs
here as a hand-written implicit-GEMM kernel on v_mfma_f32_32x32x16_bf16 — bf16 operands, fp32
accumulation, bias + ReLU fused — instead of MIOpen (whose first use of each shape also runs a
minutes-long kernel search on a fresh box).  The arithmetic is autocast's: bf16 inputs and
weights, fp32 accumulation, a bf16 result.

`MFMAConv2dReLU` is the autograd function `relu(conv2d(x, w, b))`: forward through the kernel;
backward masks the gradient with the saved output, computes the input gradient with the same
kernel (the "full" convolution of the masked gradient: implicit zero padding k - 1, the kernel
flipped and transposed) and the weight gradient with the MFMA weight-gradient kernel
(ffmp_conv2d_wgrad_bf16: positions along k through transposing LDS reads).  No MIOpen in the
loop: no per-shape kernel search on a fresh box.
"""
from __future__ import annotations

import ctypes as C
import functools
import os
from typing import Optional

import torch

from . import _abi

CONV_RELU, CONV_OUT_BF16, CONV_W_FRAG, CONV_X_FOLD = 1, 2, 4, 8  # include/ffmp.h FFMP_CONV_*


def _layer_ok(conv: torch.nn.Conv2d) -> bool:
    return (conv.stride == (1, 1) and conv.padding == (0, 0) and conv.dilation == (1, 1) and conv.groups == 1
            and conv.padding_mode == "zeros")


@functools.lru_cache(maxsize=1024)
def shape_ok(kind: int, batch: int, h: int, w: int, c: int, kh: int, kw: int, n: int, pad: int = 0, dx: int = 1) -> bool:
    """Does the kernel take this shape (include/ffmp.h ffmp_conv2d_check: the launch's own checks,
    nothing launched)?  kind 0: forward / data gradient (pad > 0), 1: weight gradient."""
    return _abi.load().ffmp_conv2d_check(kind, batch, h, w, c, kh, kw, n, pad, dx) == 0


def supported(conv: torch.nn.Conv2d, x_shape=None) -> bool:
    """Stride 1, no padding / dilation / groups, 32 or 64 channels in and out (the kernel's layers);
    with the input's NCHW shape, also every launch the layer's forward and backward make: the
    forward, the data gradient (the padded full convolution of the output gradient) and the weight
    gradient — input rows of <= 16 KiB, batch <= 65535, the LDS ring, weight-gradient rows of >= 8
    positions.  False: the caller keeps the library convolution for this shape."""
    if not (_layer_ok(conv) and conv.in_channels in (32, 64) and conv.out_channels in (32, 64)):
        return False
    if x_shape is None:
        return True
    B, C, H, W = (int(v) for v in x_shape)
    KH, KW = conv.kernel_size
    N = conv.out_channels
    Ho, Wo = H - KH + 1, W - KW + 1
    if C != conv.in_channels or Ho < 1 or Wo < 1:
        return False
    return (shape_ok(0, B, H, W, C, KH, KW, N)
            and (shape_ok(0, B, Ho, Wo, N, KH, KW, C, KH - 1) or dgrad_bm_ok(B, Ho, Wo, N, KH, KW, C))
            and shape_ok(1, B, H, W, C, KH, KW, N))


def pack_weight(w: torch.Tensor) -> torch.Tensor:
    """torch's [N][C][KH][KW] weight -> the kernel's bf16 [KH][KW][N][C]."""
    return w.detach().to(torch.bfloat16).permute(2, 3, 0, 1).contiguous()


def frag_order(wp: torch.Tensor) -> torch.Tensor:
    """A plain packed weight [KH][KW][N][C] -> the kernels' fragment order [KH][KW][N/32][C/16][2][32][8]
    (include/ffmp.h FFMP_CONV_W_FRAG: every 64-lane weight fragment load reads 1 KiB contiguous)."""
    KH, KW, N, Cc = wp.shape
    return wp.view(KH, KW, N // 32, 32, Cc // 16, 2, 8).permute(0, 1, 2, 4, 5, 3, 6).contiguous()


def small_route(h: int, w: int, c: int, kh: int, kw: int, pad: int = 0, dx: int = 1) -> bool:
    """Does ffmp_conv2d_fwd_bf16 run this shape on its small-image kernel (launch_fwd_wf's test,
    csrc/ffmp_conv.hip)?  That kernel's weight loads are ~17 % of its time faster in fragment order
    (profiles/r05sm_conv_small.txt); the row-ring kernel (conv2) gains nothing from it.  Only speed
    rides on this: both kernels take either layout, with the same results bit for bit."""
    ho, wo = h + 2 * pad - kh + 1, w + 2 * pad - (kw - 1) * dx
    if ho < 1 or wo < 1:
        return False
    cpr = 256 // (c * 2)  # lds_pitch / cell_off
    pitch = (w - 1) * c * 2 + ((w - 1) // cpr) * 16 + c * 2
    window = ((128 + wo - 1) // wo + 1 + kh - 1) * pitch + c * 2
    return ho * wo <= 2048 and kh >= 4 and window <= 76 * 1024 and (w * c * 2) % 16 == 0


def _fwd_weight(weight: torch.Tensor, kind: str, fn, h: int, w: int, c: int, kh: int, kw: int,
                pad: int = 0) -> torch.Tensor:
    """The cached kernel-layout weight for one forward launch: fragment order where the shape runs
    on the small-image kernel, else the plain layout."""
    if small_route(h, w, c, kh, kw, pad):
        return packed(weight, kind + "_frag", lambda v: frag_order(fn(v)))
    return packed(weight, kind, fn)


def pack_weight_dgrad(w: torch.Tensor) -> torch.Tensor:
    """The data gradient's kernel: w'[ky][kx][c][n] = w[n][c][KH-1-ky][KW-1-kx] (bf16)."""
    return w.detach().to(torch.bfloat16).flip(2, 3).permute(2, 3, 1, 0).contiguous()


def pack_weight_dgrad_bm(w: torch.Tensor) -> torch.Tensor:
    """ffmp_conv2d_dgrad_bf16's kernel from torch's w [N][C][KH][KW]: w'[ky][kx][n // 8][c][n % 8] =
    w[n][c][KH-1-ky][KW-1-kx] (bf16; n = the forward's output channel = the gradient's channel, in
    blocks of 8 ahead of the input channel c)."""
    N, Cc, KH, KW = w.shape
    return (w.detach().to(torch.bfloat16).flip(2, 3).view(N // 8, 8, Cc, KH, KW)
            .permute(3, 4, 0, 2, 1).contiguous())


def conv2d_dgrad_nhwc(g: torch.Tensor, w_bm: torch.Tensor, out_dtype: torch.dtype = torch.bfloat16) -> torch.Tensor:
    """dx[b, Y, X, n] = sum g[b, Y+ky-(KH-1), X+kx-(KW-1), c] w'[ky, kx, c, n] (cells outside g zero):
    the data gradient of an unpadded stride-1 convolution, 32 samples per MFMA block
    (ffmp_conv2d_dgrad_bf16).  g NHWC bf16 [B, Hy, Wy, C], w_bm from pack_weight_dgrad_bm; returns
    NHWC [B, Hy+KH-1, Wy+KW-1, N]."""
    if g.dtype != torch.bfloat16 or w_bm.dtype != torch.bfloat16:
        raise TypeError("conv2d_dgrad_nhwc takes bf16 g and packed weight")
    if not g.is_cuda or not g.is_contiguous() or not w_bm.is_contiguous():
        raise ValueError("conv2d_dgrad_nhwc takes contiguous device tensors")
    B, Hy, Wy, Cg = g.shape
    KH, KW, C8, Cn, eight = w_bm.shape
    if C8 * eight != Cg or eight != 8:
        raise ValueError(f"channel mismatch: g has {Cg}, weight {C8 * eight}")
    if out_dtype not in (torch.float32, torch.bfloat16):
        raise TypeError("out_dtype must be float32 or bfloat16")
    y = torch.empty((B, Hy + KH - 1, Wy + KW - 1, Cn), dtype=out_dtype, device=g.device)
    stream = C.c_void_p(torch.cuda.current_stream(g.device).cuda_stream)
    _abi.check(_abi.load().ffmp_conv2d_dgrad_bf16(g.data_ptr(), w_bm.data_ptr(), y.data_ptr(), B, Hy, Wy, Cg, KH, KW, Cn,
                                                  CONV_OUT_BF16 if out_dtype == torch.bfloat16 else 0, stream),
               "ffmp_conv2d_dgrad_bf16")
    return y


def dgrad_bm_ok(batch: int, hy: int, wy: int, c: int, kh: int, kw: int, n: int) -> bool:
    """Does ffmp_conv2d_dgrad_bf16 take this data gradient (c = the gradient's channels, n = the
    input's)?  FFMP_CONV_DGRAD=ring keeps every data gradient on the padded forward kernel (A/B probe)."""
    if os.environ.get("FFMP_CONV_DGRAD", "") == "ring":
        return False
    return shape_ok(2, batch, hy, wy, c, kh, kw, n)


def conv2d_nhwc(x: torch.Tensor, w_packed: torch.Tensor, bias: Optional[torch.Tensor], relu: bool = False,
                out_dtype: torch.dtype = torch.float32, pad: int = 0, dx: int = 1, x_fold: bool = False) -> torch.Tensor:
    """y[b, yo, xo, n] = act(bias[n] + sum x[b, yo+ky, xo+kx*dx, c] w[ky, kx, n, c]) for an NHWC
    bf16 x [B, H, W, C] (zero-padded by `pad` cells on every side) and a packed weight
    [KH, KW, N, C] (or the same in fragment order, frag_order's 7-d [KH, KW, N/32, C/16, 2, 32, 8]);
    returns NHWC [B, H+2pad-KH+1, W+2pad-(KW-1)dx, N].  x_fold: x is the unfolded [B, H, W + dx - 1,
    C / dx] input whose fold_input(., dx) the kernel reads on the fly (FFMP_CONV_X_FOLD)."""
    if x.dtype != torch.bfloat16 or w_packed.dtype != torch.bfloat16:
        raise TypeError("conv2d_nhwc takes bf16 x and packed weight")
    if not x.is_cuda or not x.is_contiguous() or not w_packed.is_contiguous():
        raise ValueError("conv2d_nhwc takes contiguous device tensors")
    B, H, W, Cin = x.shape
    if x_fold:  # the folded image the kernel sees
        W, Cin = W - dx + 1, Cin * dx
    frag = w_packed.dim() == 7
    if frag:
        KH, KW, NB, S, two, r32, e8 = w_packed.shape
        if (two, r32, e8) != (2, 32, 8):
            raise ValueError(f"fragment-order weight must end in (2, 32, 8), got {tuple(w_packed.shape)}")
        N, Cw = NB * 32, S * 16
    else:
        KH, KW, N, Cw = w_packed.shape
    if Cw != Cin:
        raise ValueError(f"channel mismatch: x has {Cin}, weight {Cw}")
    if out_dtype not in (torch.float32, torch.bfloat16):
        raise TypeError("out_dtype must be float32 or bfloat16")
    y = torch.empty((B, H + 2 * pad - KH + 1, W + 2 * pad - (KW - 1) * dx, N), dtype=out_dtype, device=x.device)
    b = None
    if bias is not None:
        b = bias.detach().to(device=x.device, dtype=torch.float32).contiguous()
    flags = (CONV_RELU if relu else 0) | (CONV_OUT_BF16 if out_dtype == torch.bfloat16 else 0) | \
        (CONV_W_FRAG if frag else 0) | (CONV_X_FOLD if x_fold else 0)
    lib = _abi.load()
    stream = C.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)
    _abi.check(lib.ffmp_conv2d_fwd_bf16(x.data_ptr(), w_packed.data_ptr(), None if b is None else b.data_ptr(),
                                        y.data_ptr(), B, H, W, Cin, KH, KW, N, int(pad), int(dx), flags, stream),
               "ffmp_conv2d_fwd_bf16")
    return y


def conv2d_wgrad_nhwc(g: torch.Tensor, x: torch.Tensor, KH: int, KW: int, dx: int = 1,
                      chunks: Optional[int] = None) -> torch.Tensor:
    """dW[ky, kx, n, c] = sum_{b, p} g[b, p, n] x[b, yp+ky, xp+kx*dx, c] (fp32) for NHWC bf16 g
    [B, Ho, Wo, N] and x [B, H, W, C]: the MFMA weight-gradient kernel's per-chunk partials, summed."""
    if g.dtype != torch.bfloat16 or x.dtype != torch.bfloat16:
        raise TypeError("conv2d_wgrad_nhwc takes bf16 g and x")
    if not (g.is_contiguous() and x.is_contiguous() and g.is_cuda and x.is_cuda):
        raise ValueError("conv2d_wgrad_nhwc takes contiguous device tensors")
    B, H, W, Cin = x.shape
    Bg, Ho, Wo, N = g.shape
    if Bg != B or Ho != H - KH + 1 or Wo != W - (KW - 1) * dx:
        raise ValueError(f"shape mismatch: g {tuple(g.shape)}, x {tuple(x.shape)}, kernel {KH}x{KW} dx {dx}")
    if chunks is None:  # ~512 workgroups (taps per workgroup: 32 at 32 -> 64 channels, else 8)
        groups = KH * KW // (32 if (Cin, N) == (32, 64) else 8)
        chunks = max(1, min(B, 512 // max(groups, 1)))
    part = torch.empty((chunks, KH, KW, N, Cin), dtype=torch.float32, device=g.device)
    stream = C.c_void_p(torch.cuda.current_stream(g.device).cuda_stream)
    _abi.check(_abi.load().ffmp_conv2d_wgrad_bf16(g.data_ptr(), x.data_ptr(), part.data_ptr(), B, H, W, Cin, KH, KW, N,
                                                  int(dx), int(chunks), stream), "ffmp_conv2d_wgrad_bf16")
    return part.sum(0) if chunks > 1 else part[0]


def _bump_versions(optimizer: torch.optim.Optimizer, args, kwargs) -> None:
    """Optimizer step post-hook: mark every parameter of the optimizer as written in place."""
    torch.autograd.graph.increment_version([p for g in optimizer.param_groups for p in g["params"]])


def track_optimizer(optimizer: torch.optim.Optimizer):
    """Keep `packed`'s weight caches honest under an optimizer that writes parameters without
    bumping their version counter.  torch's fused Adam (fused=True) and the other fused/foreach
    kernels update the storage in place through a raw kernel: p._version stays unchanged and the
    data_ptr too, so a cached bf16 pack would outlive the update.  This installs a step post-hook
    that bumps every parameter's version after each step(); returns the hook handle.  Brain does
    this for its own optimizer; any other optimizer driving an MFMA Network must too."""
    return optimizer.register_step_post_hook(_bump_versions)


def packed(weight: torch.Tensor, kind: str, fn) -> torch.Tensor:
    """fn(weight) — a kernel-layout copy of a layer's weight — cached on the weight tensor until the
    weight changes (its in-place version counter: load_state_dict's copy_ and autograd-visible
    in-place ops bump it; a fused optimizer does NOT — see track_optimizer).  One training step runs
    the online network three times (acting, Q(s), Q(s')) and packs its weights once; the target
    network's packs live until the next sync."""
    stamp = (weight._version, weight.data_ptr())
    cache = getattr(weight, "_ffmp_packs", None)
    if cache is None:
        cache = {}
        try:
            weight._ffmp_packs = cache
        except (AttributeError, RuntimeError):  # a tensor that takes no attributes: no cache
            return fn(weight)
    hit = cache.get(kind)
    if hit is not None and hit[0] == stamp:
        return hit[1]
    v = fn(weight)
    cache[kind] = (stamp, v)
    return v


def relu_masked_nhwc(gy: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """The ReLU's backward in one kernel: gy (NCHW-shaped, channels-last strides) where the NHWC
    output y > 0, else 0, as a contiguous bf16 NHWC tensor."""
    g = gy.permute(0, 2, 3, 1)
    if g.dtype != torch.bfloat16:
        g = g.to(torch.bfloat16)
    return torch.ops.aten.threshold_backward(g, y, 0).contiguous()


class MFMAConv2dReLU(torch.autograd.Function):
    """relu(conv2d(x, weight, bias)) in bf16 with fp32 accumulation; returns a bf16 NCHW-shaped
    tensor (channels-last strides).  The bias is added in fp32 (autocast's conv2d rounds it to
    bf16 first: a difference of at most half a bf16 ulp of the bias)."""

    @staticmethod
    def forward(ctx, x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor]):
        xb = x.to(torch.bfloat16).permute(0, 2, 3, 1).contiguous()  # NHWC (free if x is channels-last)
        KH, KW = weight.shape[2], weight.shape[3]
        wb = _fwd_weight(weight, "fwd", pack_weight, xb.shape[1], xb.shape[2], xb.shape[3], KH, KW)
        y = conv2d_nhwc(xb, wb, bias, relu=True, out_dtype=torch.bfloat16)
        ctx.save_for_backward(xb, weight, y)
        ctx.has_bias = bias is not None
        ctx.x_dtype = x.dtype
        return y.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, gy: torch.Tensor):
        xb, weight, y = ctx.saved_tensors
        g = relu_masked_nhwc(gy, y)  # NHWC, masked by the ReLU
        need = ctx.needs_input_grad
        gx = gw = gb = None
        if need[0]:  # the full convolution of g with the flipped, transposed kernel, on the matrix cores
            N, Cin, KH, KW = weight.shape
            B, Hy, Wy, _ = g.shape
            if dgrad_bm_ok(B, Hy, Wy, N, KH, KW, Cin):  # 32 samples per MFMA block: no zero products
                gx = conv2d_dgrad_nhwc(g, packed(weight, "dgrad_bm", pack_weight_dgrad_bm))
            else:
                wd = _fwd_weight(weight, "dgrad", pack_weight_dgrad, Hy, Wy, N, KH, KW, KH - 1)
                gx = conv2d_nhwc(g, wd, None, out_dtype=torch.bfloat16, pad=KH - 1)
            gx = gx.permute(0, 3, 1, 2).to(ctx.x_dtype)
        if need[1]:  # on the matrix cores too: [KH][KW][N][C] -> torch's [N][C][KH][KW]
            gw = conv2d_wgrad_nhwc(g, xb, weight.shape[2], weight.shape[3]).permute(2, 3, 0, 1).to(weight.dtype)
        if ctx.has_bias and need[2]:
            gb = g.sum((0, 1, 2), dtype=torch.float32)  # fp32 accumulation, no fp32 copy of g
        return gx, gw, gb


def conv_relu(conv: torch.nn.Conv2d, x: torch.Tensor) -> torch.Tensor:
    """relu(conv(x)) through the MFMA kernel (bf16, as under autocast)."""
    return MFMAConv2dReLU.apply(x, conv.weight, conv.bias)


# ---------------------------------------------------------------- few-channel inputs (conv1)
# conv1 = nn.Conv2d(2, 32, kernel_size=32) (train.py:234) reads 2 channels: a K step of 16 would be
# mostly padding.  Folding F = 32 / C consecutive kernel columns into the channel axis —
# x'[b, y, x, j*C + c] = x[b, c, y, x + j], w'[ky, kx', n, j*C + c] = w[n, c, ky, kx'*F + j] —
# turns it into a 32-channel convolution with KW / F kernel columns read F cells apart (dx = F):
#   y[b, yo, xo, n] = sum_{ky, kx', q} x'[b, yo+ky, xo+kx'*F, q] w'[ky, kx', n, q]
# the same products and sum as the original, on the MFMA kernel.

def fold_channels(c: int) -> int:
    """The channels a c-channel input is zero-padded to before folding: the next power of two
    (3 -> 4, 12 -> 16), so F = 32 / that kernel columns fill the 32 folded channels."""
    return 1 << (int(c) - 1).bit_length()


def fold_supported(conv: torch.nn.Conv2d, x_shape=None) -> bool:
    """A 1-16 channel layer whose kernel width folds into 32 channels (padded to a power of two:
    the reference's 1 / 2 / 3 map channels and the 12-channel BEV series); with the input's NCHW
    shape, also the folded forward and weight-gradient launches (the input gradient is MIOpen's)."""
    c = conv.in_channels
    if not (_layer_ok(conv) and 1 <= c <= 16 and conv.kernel_size[1] % (32 // fold_channels(c)) == 0
            and conv.out_channels in (32, 64)):
        return False
    if x_shape is None:
        return True
    B, Cx, H, W = (int(v) for v in x_shape)
    KH, KW = conv.kernel_size
    F = 32 // fold_channels(c)
    if Cx != c or H < KH or W < KW:
        return False
    return (shape_ok(0, B, H, W - F + 1, 32, KH, KW // F, conv.out_channels, 0, F)
            and shape_ok(1, B, H, W - F + 1, 32, KH, KW // F, conv.out_channels, 0, F))


def nhwc_bf16(x: torch.Tensor) -> torch.Tensor:
    """x (B, C, H, W), any dtype / strides -> a contiguous bf16 NHWC copy, in one kernel (cast and
    transpose together)."""
    B, Cc, H, W = x.shape
    return torch.empty((B, H, W, Cc), dtype=torch.bfloat16, device=x.device).copy_(x.permute(0, 2, 3, 1))


def fold_input(x: torch.Tensor, F: int) -> torch.Tensor:
    """x (B, C, H, W) -> bf16 NHWC (B, H, W - F + 1, F * C) with channel j*C + c = x[:, c, :, x + j]."""
    B, Cc, H, W = x.shape
    xn = nhwc_bf16(x)  # (B, H, W, C)
    s = xn.stride()
    v = xn.as_strided((B, H, W - F + 1, F, Cc), (s[0], s[1], s[2], s[2], s[3]))
    return v.reshape(B, H, W - F + 1, F * Cc).contiguous()


def pack_weight_fold(w: torch.Tensor, F: int) -> torch.Tensor:
    """w (N, C, KH, KW) -> bf16 (KH, KW / F, N, F * C) with channel j*C + c = w[n, c, ky, kx'*F + j]."""
    N, Cc, KH, KW = w.shape
    v = w.detach().to(torch.bfloat16).view(N, Cc, KH, KW // F, F)       # [n, c, ky, kx', j]
    return v.permute(2, 3, 0, 4, 1).reshape(KH, KW // F, N, F * Cc).contiguous()


class MFMAFoldConv2dReLU(torch.autograd.Function):
    """relu(conv2d(x, weight, bias)) for a 1/2/4/8/16-channel x on the MFMA kernel (kernel columns folded
    into 32 channels); bf16 NCHW-shaped result (channels-last strides).  Backward: the weight
    gradient of the folded convolution on the MFMA kernel, unfolded; the input's (MIOpen) only if
    asked for."""

    @staticmethod
    def forward(ctx, x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor]):
        F = 32 // x.shape[1]
        # fragment-order weights: 0-3 % faster at B = 256 (profiles/r05fab_conv_frag_ab.txt, r05sf_learner.txt)
        wf = packed(weight, f"fold{F}_frag", lambda v: frag_order(pack_weight_fold(v, F)))
        if x.shape[1] % 2 == 0:  # the kernel folds the NHWC input on the fly (dword cells: >= 2 channels)
            y = conv2d_nhwc(nhwc_bf16(x), wf, bias, relu=True, out_dtype=torch.bfloat16, dx=F, x_fold=True)
        else:
            y = conv2d_nhwc(fold_input(x, F), wf, bias, relu=True, out_dtype=torch.bfloat16, dx=F)
        ctx.save_for_backward(x, weight, y)
        ctx.has_bias = bias is not None
        return y.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, gy: torch.Tensor):
        x, weight, y = ctx.saved_tensors
        g = relu_masked_nhwc(gy, y)  # NHWC
        need = ctx.needs_input_grad
        gx = gw = gb = None
        if need[0]:  # the map input has no gradient in the Network; for completeness, MIOpen's
            wt = weight.detach().to(torch.bfloat16)
            gx = torch.ops.aten.convolution_backward(g.permute(0, 3, 1, 2), x.to(torch.bfloat16), wt, None, [1, 1],
                                                     [0, 0], [1, 1], False, [0, 0], 1, [True, False, False])[0]
            gx = gx.to(x.dtype)
        if need[1]:  # the folded kernel's weight gradient, unfolded: q = j * C + c, kx = kx' * F + j
            N, Cc, KH, KW = weight.shape
            F = 32 // Cc
            gwf = conv2d_wgrad_nhwc(g, fold_input(x, F), KH, KW // F, dx=F)  # [KH][KW/F][N][F*C]
            gw = gwf.view(KH, KW // F, N, F, Cc).permute(2, 4, 0, 1, 3).reshape(N, Cc, KH, KW).to(weight.dtype)
        if ctx.has_bias and need[2]:
            gb = g.sum((0, 1, 2), dtype=torch.float32)  # fp32 accumulation, no fp32 copy of g
        return gx, gw, gb


def fold_conv_relu(conv: torch.nn.Conv2d, x: torch.Tensor) -> torch.Tensor:
    """relu(conv(x)) for a few-channel conv (the reference's conv1) through the MFMA kernel."""
    w = conv.weight
    pad = fold_channels(x.shape[1]) - x.shape[1]
    if pad:  # zero channels (zero products): 3 -> 4 keeps the fold at F = 8 columns, 12 -> 16 at F = 2
        x = torch.nn.functional.pad(x, (0, 0, 0, 0, 0, pad))
        w = torch.nn.functional.pad(w, (0, 0, 0, 0, 0, pad))
    return MFMAFoldConv2dReLU.apply(x, w, conv.bias)
