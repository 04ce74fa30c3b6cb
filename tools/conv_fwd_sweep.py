#!/usr/bin/env python3
"""conv2's MFMA forward (32 -> 64, k = 32, 69^2 -> 38^2, bf16 out + ReLU, as the Network runs it) over a
list of batch sizes: TFLOP/s per B, to see the workgroup-count quantisation (3 tiles of 512 positions
per sample, 2 workgroups per CU: B = 170 fills the chip once, 256 one and a half times).
Usage: python tools/conv_fwd_sweep.py [B ...]   (FFMP_CONV_MBW=1/2/4 forces the tile)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flow_field_based_motion_planner_amd.conv_mfma import conv2d_nhwc, pack_weight  # noqa: E402

dev = torch.device("cuda:0")


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


w = (torch.randn(64, 32, 32, 32, device=dev) / 181.0).to(torch.bfloat16)
wp = pack_weight(w)
if os.environ.get("FFMP_SWEEP_WFRAG"):  # probe builds reading B in fragment order: [tap][nb][s][h][r][8]
    KH, KW, N, C = wp.shape
    wp = wp.view(KH * KW, N // 32, 32, C // 16, 2, 8).permute(0, 1, 3, 4, 2, 5).contiguous().view(KH, KW, N, C)
bias = torch.randn(64, device=dev)
for B in [int(a) for a in (sys.argv[1:] or ["128", "170", "171", "256", "340", "342", "512", "1024"])]:
    xn = torch.relu(torch.randn(B, 69, 69, 32, device=dev)).to(torch.bfloat16)
    ms = timeit(lambda: conv2d_nhwc(xn, wp, bias, relu=True, out_dtype=torch.bfloat16))
    flop = 2.0 * B * 38 * 38 * 64 * 32 * 32 * 32
    print(f"MBW={os.environ.get('FFMP_CONV_MBW', 'auto')} B={B:5d}: {ms:.3f} ms {flop / ms / 1e9:7.1f} TFLOP/s "
          f"({ms / B * 1e3:.2f} us/sample)", flush=True)
