#!/usr/bin/env python3
"""The learner's MFMA convolutions at B = 256 (the reference Network's shapes at the 100^2 map), HIP
events, median of 3 x 10 launches: conv2 forward / data gradient / weight gradient, conv1 folded,
conv3 + conv4 (small-image kernel) forward and data gradient.  TFLOP/s counts the useful products
(2 x outputs x taps x input channels).  Launch knobs come from the environment (FFMP_CONV_MBW)."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flow_field_based_motion_planner_amd.conv_mfma import (conv2d_nhwc, conv2d_wgrad_nhwc, fold_input,  # noqa: E402
                                                          pack_weight, pack_weight_dgrad, pack_weight_fold)

dev = torch.device("cuda:0")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 256


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1) / reps)
    return statistics.median(out)


def shape(cin, cout, hin, k):
    ho = hin - k + 1
    x = torch.relu(torch.randn(B, hin, hin, cin, device=dev)).to(torch.bfloat16).contiguous()
    w = (torch.randn(cout, cin, k, k, device=dev) / (k * cin ** 0.5)).to(torch.bfloat16)
    g = torch.randn(B, ho, ho, cout, device=dev).to(torch.bfloat16).contiguous()
    return x, w, g, 2.0 * B * ho * ho * cout * cin * k * k


rows = []
x, w, g, fl = shape(32, 64, 69, 32)  # conv2
wp, wd = pack_weight(w), pack_weight_dgrad(w)
rows.append(("conv2 fwd", timeit(lambda: conv2d_nhwc(x, wp, None, relu=True, out_dtype=torch.bfloat16)), fl))
rows.append(("conv2 dgrad", timeit(lambda: conv2d_nhwc(g, wd, None, out_dtype=torch.bfloat16, pad=31)), fl))
rows.append(("conv2 wgrad", timeit(lambda: conv2d_wgrad_nhwc(g, x, 32, 32)), fl))
x3, w3, g3, fl3 = shape(64, 64, 38, 8)  # conv3
rows.append(("conv3 fwd", timeit(lambda: conv2d_nhwc(x3, pack_weight(w3), None, relu=True, out_dtype=torch.bfloat16)), fl3))
rows.append(("conv3 dgrad", timeit(lambda: conv2d_nhwc(g3, pack_weight_dgrad(w3), None, out_dtype=torch.bfloat16, pad=7)), fl3))
rows.append(("conv3 wgrad", timeit(lambda: conv2d_wgrad_nhwc(g3, x3, 8, 8)), fl3))
s0 = (torch.rand(B, 2, 100, 100, device=dev) > 0.9).float() * 255
w1 = torch.randn(32, 2, 32, 32, device=dev) / 45.0
w1f = pack_weight_fold(w1, 16)
fl1 = 2.0 * B * 69 * 69 * 32 * 2 * 32 * 32
rows.append(("conv1 fold fwd", timeit(lambda: conv2d_nhwc(fold_input(s0, 16), w1f, None, relu=True,
                                                          out_dtype=torch.bfloat16, dx=16)), fl1))
tag = os.environ.get("FFMP_CONV_MBW", "auto")
for name, ms, f in rows:
    print(f"mbw={tag:4s} B={B} {name:16s} {ms:8.3f} ms  {f / ms / 1e9:7.1f} TFLOP/s useful", flush=True)
