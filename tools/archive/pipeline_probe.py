#!/usr/bin/env python3
"""The two-launch C3 step with its env kernel split into S slices on a side stream, each slice's
raster on the main stream as soon as its env slice is done (FFMPVec(pipeline=S)), vs S = 1: whole-step
ms over 3 x 24 steps per variant, alternating, one instance per variant (autotuned)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flow_field_based_motion_planner_amd.vec_env import FFMPVec  # noqa: E402

dev = torch.device("cuda:0")
a = torch.full((32768,), 10, dtype=torch.int64, device=dev)
env = FFMPVec(32768, "C3", device=dev, fused=False)
print("shape", env.raster_shape_newest, flush=True)
tun = env.tuning()
for rep in range(3):
    for S in (1, 2, 4, 8):
        env.pipeline_slices = S
        env._build_slices()
        env.reset()
        for _ in range(8):
            env.step(a)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(24):
            env.step(a)
        e1.record()
        torch.cuda.synchronize()
        print(f"rep {rep} S={S} step {e0.elapsed_time(e1) / 24:.4f} ms", flush=True)
