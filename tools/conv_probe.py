#!/usr/bin/env python3
"""Time the reference Network's conv2 (32 -> 64, k = 32, 69^2 -> 38^2) at batch B: the MFMA kernel
(ffmp_conv2d_fwd_bf16) against MIOpen bf16 (NCHW, channels-last; cudnn.benchmark), forward, and
MIOpen's data / weight gradients for scale.  TFLOP/s = 2 * B * 38^2 * 64 * 32 * 32^2 / time."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flow_field_based_motion_planner_amd.conv_mfma import (conv2d_dgrad_nhwc, conv2d_nhwc, conv2d_wgrad_nhwc,  # noqa: E402
                                                          fold_input, pack_weight, pack_weight_dgrad,
                                                          pack_weight_dgrad_bm, pack_weight_fold)

dev = torch.device("cuda:0")
torch.backends.cudnn.benchmark = True


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


MFMA_ONLY = "--mfma-only" in sys.argv  # skip the MIOpen rows (their searches take minutes on a fresh box)
for B in [int(a) for a in ([a for a in sys.argv[1:] if not a.startswith("--")] or ["256", "1024"])]:
    flop = 2.0 * B * 38 * 38 * 64 * 32 * 32 * 32
    x = torch.relu(torch.randn(B, 32, 69, 69, device=dev)).to(torch.bfloat16)
    w = (torch.randn(64, 32, 32, 32, device=dev) / 181.0).to(torch.bfloat16)
    bias = torch.randn(64, device=dev)
    xn = x.permute(0, 2, 3, 1).contiguous()
    wp = pack_weight(w)
    xcl = x.contiguous(memory_format=torch.channels_last)
    rows = {}
    rows["mfma fwd (bf16 out, relu)"] = timeit(lambda: conv2d_nhwc(xn, wp, bias, relu=True, out_dtype=torch.bfloat16))
    rows["mfma fwd (f32 out)"] = timeit(lambda: conv2d_nhwc(xn, wp, bias))
    if not MFMA_ONLY:
        rows["miopen fwd NCHW"] = timeit(lambda: F.conv2d(x, w, bias.to(torch.bfloat16)))
        rows["miopen fwd NHWC"] = timeit(lambda: F.conv2d(xcl, w.contiguous(memory_format=torch.channels_last),
                                                          bias.to(torch.bfloat16)))
    gy = torch.randn(B, 64, 38, 38, device=dev).to(torch.bfloat16)
    gn = gy.permute(0, 2, 3, 1).contiguous()
    wd = pack_weight_dgrad(w)
    rows["mfma dgrad (pad 31, bf16 out)"] = timeit(lambda: conv2d_nhwc(gn, wd, None, out_dtype=torch.bfloat16, pad=31))
    wbm = pack_weight_dgrad_bm(w)
    rows["mfma dgrad bm (bf16 out)"] = timeit(lambda: conv2d_dgrad_nhwc(gn, wbm))
    if not MFMA_ONLY:
        rows["miopen dgrad NCHW"] = timeit(lambda: torch.ops.aten.convolution_backward(
            gy, x, w, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1, [True, False, False]))
    rows["mfma wgrad"] = timeit(lambda: conv2d_wgrad_nhwc(gn, xn, 32, 32))
    if not MFMA_ONLY:
        rows["miopen wgrad NCHW"] = timeit(lambda: torch.ops.aten.convolution_backward(
            gy, x, w, [64], [1, 1], [0, 0], [1, 1], False, [0, 0], 1, [False, True, True]))
    for k, ms in rows.items():
        print(f"B={B:5d} {k:28s} {ms:8.3f} ms  {flop / ms / 1e9:7.1f} TFLOP/s", flush=True)
    # conv1: 2 -> 32 channels, k = 32, 100^2 -> 69^2 (0.62 GFLOP per sample)
    flop1 = 2.0 * B * 69 * 69 * 32 * 2 * 32 * 32
    s0 = (torch.rand(B, 2, 100, 100, device=dev) > 0.9).float() * 255
    w1 = torch.randn(32, 2, 32, 32, device=dev) / 45.0
    w1f = pack_weight_fold(w1, 16)
    r1 = {"mfma conv1 fold (incl. fold)": timeit(lambda: conv2d_nhwc(fold_input(s0, 16), w1f, None, relu=True,
                                                                      out_dtype=torch.bfloat16, dx=16)),
          }
    if not MFMA_ONLY:
        r1["miopen conv1 fwd NCHW"] = timeit(lambda: F.conv2d(s0.to(torch.bfloat16), w1.to(torch.bfloat16)))
    for k, ms in r1.items():
        print(f"B={B:5d} {k:28s} {ms:8.3f} ms  {flop1 / ms / 1e9:7.1f} TFLOP/s", flush=True)
