#!/usr/bin/env python3
"""Debug: the MFMA weight-gradient kernel on one-hot inputs (KH=8, KW=1, C=N=32, one output row of
16 positions): which (tap, n, c) entries a single g or x element reaches."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flow_field_based_motion_planner_amd.conv_mfma import conv2d_wgrad_nhwc  # noqa: E402

dev = "cuda:0"
B, H, W, C, KH, KW, N = 1, 8, 16, 32, 8, 1, 32
Ho, Wo = 1, 16
x1 = torch.ones((B, H, W, C), device=dev, dtype=torch.bfloat16)
for p in (0, 1, 3, 4, 7, 8, 15):
    for n in (0, 5, 31):
        g = torch.zeros((B, Ho, Wo, N), device=dev, dtype=torch.bfloat16)
        g[0, 0, p, n] = 1.0
        dw = conv2d_wgrad_nhwc(g, x1, KH, KW, chunks=1)  # want dw[ky, 0, n, c] = 1 for all ky, c
        nz = dw[0, 0].nonzero().tolist()
        print(f"g one-hot p={p:2d} n={n:2d}: tap0 sum {float(dw[0,0].sum()):6.1f} nonzero rows(n) "
              f"{sorted(set(a for a, b in nz))} vals {sorted(set(float(dw[0,0][a,b]) for a, b in nz))}")
g1 = torch.ones((B, Ho, Wo, N), device=dev, dtype=torch.bfloat16)
for yy, xx, c in ((0, 0, 0), (0, 3, 7), (2, 5, 0), (7, 15, 31)):
    x = torch.zeros((B, H, W, C), device=dev, dtype=torch.bfloat16)
    x[0, yy, xx, c] = 1.0
    dw = conv2d_wgrad_nhwc(g1, x, KH, KW, chunks=1)  # want dw[yy, 0, n, c] = 1 for all n
    nz = dw.nonzero().tolist()
    print(f"x one-hot y={yy} x={xx} c={c}: taps {sorted(set(a for a, *_ in nz))} cols {sorted(set(d for *_, d in nz))} "
          f"vals {sorted(set(float(dw[tuple(t)]) for t in nz))}")
