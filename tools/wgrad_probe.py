"""Time the conv2 weight gradient (32 -> 64 channels, k = 32, 69^2 -> 38^2, B = 256) on the MFMA kernel
for several batch-chunk counts; TFLOP/s = 2 B 38^2 64 32 32^2 / time.  usage: wgrad_probe.py [chunks ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flow_field_based_motion_planner_amd.conv_mfma import conv2d_wgrad_nhwc  # noqa: E402

dev = torch.device("cuda:0")
B = 256
flop = 2.0 * B * 38 * 38 * 64 * 32 * 32 * 32
x = torch.relu(torch.randn(B, 69, 69, 32, device=dev)).to(torch.bfloat16)
g = torch.randn(B, 38, 38, 64, device=dev).to(torch.bfloat16)
for chunks in [int(a) for a in sys.argv[1:]] or [None]:
    fn = lambda: conv2d_wgrad_nhwc(g, x, 32, 32, chunks=chunks)  # noqa: E731
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(f"chunks {chunks}: wgrad {ms:.3f} ms  {flop / ms / 1e9:.1f} TFLOP/s", flush=True)
