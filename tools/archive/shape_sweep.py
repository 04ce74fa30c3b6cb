#!/usr/bin/env python3
"""Steady-state raster ms per launch at C3 (two-launch step, one instance) for candidate launch shapes
beyond the autotune's list: 24 steps per shape after 8 untimed ones, two passes."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flow_field_based_motion_planner_amd import _abi  # noqa: E402
from flow_field_based_motion_planner_amd.vec_env import FFMPVec  # noqa: E402

NT, PL, XCD = _abi.RASTER_NT, _abi.RASTER_PLAIN, _abi.RASTER_XCD
T2, T4, T8 = _abi.RASTER_TILE2, _abi.RASTER_TILE4, _abi.RASTER_TILE8
SHAPES = [(4096, NT | XCD | T4), (2048, NT | XCD | T4), (3072, NT | XCD | T4), (4096, NT | XCD | T8),
          (4096, PL | XCD | T4), (6144, NT | XCD | T4), (8192, NT | XCD | T4), (4096, NT | T4), (2048, NT | XCD | T8)]
dev = torch.device("cuda:0")
env = FFMPVec(32768, "C3", device=dev, fused=False)
print("autotune chose", env.raster_shape_newest, flush=True)
a = torch.full((32768,), 10, dtype=torch.int64, device=dev)
env.reset()
for rep in range(2):
    for sh in SHAPES:
        env.raster_shape = env.raster_shape_newest = sh
        for _ in range(8):
            env.step(a)
        t = []
        for _ in range(24):
            env.step(a, timing=t)
        torch.cuda.synchronize()
        ms = [r[0].elapsed_time(r[1]) for r in t]
        print(f"rep {rep} {sh[0]:6d}/{sh[1]:3d} steady {sum(ms) / len(ms):.3f} ms", flush=True)
