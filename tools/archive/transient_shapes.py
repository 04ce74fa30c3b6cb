#!/usr/bin/env python3
"""Which raster launch shapes run slow for the first steps after the GPU idled?  One C3 FFMPVec
(two-launch step), then per shape: 0.5 s of host sleep, reset(), 24 steps; per-launch raster ms."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flow_field_based_motion_planner_amd import _abi  # noqa: E402
from flow_field_based_motion_planner_amd.vec_env import FFMPVec  # noqa: E402

NT, XCD, T4, T2 = _abi.RASTER_NT, _abi.RASTER_XCD, _abi.RASTER_TILE4, _abi.RASTER_TILE2
SHAPES = [(4096, NT | T4), (4096, NT | XCD | T4), (8192, NT | T4), (8192, NT | XCD | T4), (16384, NT | T4),
          (16384, NT | XCD | T4), (8192, NT | T2), (8192, NT | XCD | T2)]
dev = torch.device("cuda:0")
env = FFMPVec(32768, "C3", device=dev, fused=False)
print("autotune chose", env.raster_shape_newest, flush=True)
a = torch.full((32768,), 10, dtype=torch.int64, device=dev)
for rep in range(2):
    for sh in SHAPES:
        env.raster_shape = env.raster_shape_newest = sh
        torch.cuda.synchronize()
        time.sleep(0.5)
        env.reset()
        t = []
        for _ in range(24):
            env.step(a, timing=t)
        torch.cuda.synchronize()
        ms = [r[0].elapsed_time(r[1]) for r in t]
        print(f"{sh[0]:6d}/{sh[1]:3d} first8 " + " ".join(f"{x:.2f}" for x in ms[:8]) +
              f" | steady {sum(ms[12:]) / len(ms[12:]):.3f}", flush=True)
