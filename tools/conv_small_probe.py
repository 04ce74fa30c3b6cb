"""The Network's conv3 / conv4 forwards (64 -> 64 channels, 8 x 8 kernels: 38^2 -> 31^2 -> 24^2 ->
17^2 -> 10^2) at B = 256 on the MFMA kernels, per shape.  With the probe build of tools/gpu_r04y.sh
(FFMP_LIB=tools/_build/libffmp_sm.so), FFMP_CONV_SMALL_MAX (read once per process) moves shapes
between conv_small_kernel and the row-ring conv_fwd_kernel; the shipped library ignores it."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flow_field_based_motion_planner_amd.conv_mfma import conv2d_nhwc, pack_weight  # noqa: E402

dev = torch.device("cuda:0")
B = 256
w0 = (torch.randn(64, 64, 8, 8, device=dev) / 64.0).to(torch.bfloat16)
w = pack_weight(w0)
if os.environ.get("FFMP_SWEEP_WFRAG"):  # probe builds reading B in fragment order: [tap][nb][s][h][r][8]
    KH, KW, N, C = w.shape
    w = w.view(KH * KW, N // 32, 32, C // 16, 2, 8).permute(0, 1, 3, 4, 2, 5).contiguous().view(KH, KW, N, C)
bias = torch.randn(64, device=dev)
tag = os.environ.get("FFMP_CONV_SMALL_MAX", "2048")
tot = 0.0
for H in (38, 31, 24, 17):
    x = torch.relu(torch.randn(B, H, H, 64, device=dev)).to(torch.bfloat16)
    fn = lambda: conv2d_nhwc(x, w, bias, relu=True, out_dtype=torch.bfloat16)  # noqa: E731
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    ref = torch.relu(torch.nn.functional.conv2d(x[:8].permute(0, 3, 1, 2).float(), w0.float(), bias))
    err = (fn()[:8].float() - ref.permute(0, 2, 3, 1)).abs().max().item()
    Ho = H - 7
    flop = 2.0 * B * Ho * Ho * 64 * 64 * 64
    tot += ms
    print(f"small_max {tag}: {H}^2 -> {Ho}^2  {ms:.4f} ms  {flop / ms / 1e9:.0f} TFLOP/s  maxerr {err:.3g}", flush=True)
print(f"small_max {tag}: the four shapes {tot:.4f} ms", flush=True)
