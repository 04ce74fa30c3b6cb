"""Plain vs fragment-order weights (include/ffmp.h FFMP_CONV_W_FRAG) on every forward-kernel launch
of the Network's learner step at B = 256: the folded conv1, conv2, conv3 / conv4 (the small-image
kernel) and the data gradients of conv3 / conv4 (pad 7).  Same process, alternating, 3 rounds;
the outputs of the two layouts are compared bit for bit.
usage: python tools/conv_frag_ab.py [B]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flow_field_based_motion_planner_amd.conv_mfma import (conv2d_nhwc, frag_order, pack_weight,  # noqa: E402
                                                          small_route)

dev = torch.device("cuda:0")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
# (name, H, W, C, KH, KW, N, pad, dx)
shapes = [("conv1 fold", 100, 85, 32, 32, 2, 32, 0, 16), ("conv2", 69, 69, 32, 32, 32, 64, 0, 1),
          ("conv3", 38, 38, 64, 8, 8, 64, 0, 1), ("conv4a", 31, 31, 64, 8, 8, 64, 0, 1),
          ("conv4b", 24, 24, 64, 8, 8, 64, 0, 1), ("conv4c", 17, 17, 64, 8, 8, 64, 0, 1),
          ("dgrad conv4c", 10, 10, 64, 8, 8, 64, 7, 1), ("dgrad conv3", 31, 31, 64, 8, 8, 64, 7, 1)]


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for name, H, W, Cc, KH, KW, N, pad, dx in shapes:
    x = torch.relu(torch.randn(B, H, W, Cc, device=dev)).to(torch.bfloat16)
    wp = pack_weight(torch.randn(N, Cc, KH, KW, device=dev) / (Cc * KH * KW) ** 0.5)
    wf = frag_order(wp)
    plain = lambda: conv2d_nhwc(x, wp, None, relu=True, out_dtype=torch.bfloat16, pad=pad, dx=dx)  # noqa: E731
    frag = lambda: conv2d_nhwc(x, wf, None, relu=True, out_dtype=torch.bfloat16, pad=pad, dx=dx)  # noqa: E731
    assert torch.equal(plain(), frag()), name
    tp, tf = [], []
    for _ in range(3):
        tp.append(timeit(plain))
        tf.append(timeit(frag))
    print(f"{name:13s} small_route={int(small_route(H, W, Cc, KH, KW, pad, dx))}  plain "
          f"{' '.join(f'{t:7.1f}' for t in tp)} us   frag {' '.join(f'{t:7.1f}' for t in tf)} us", flush=True)
