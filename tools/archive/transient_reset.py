#!/usr/bin/env python3
"""Is the slow start after reset() a property of the episodes (random actions, as bench.py's) or of the
GPU's state?  One C3 FFMPVec with the 4096-cell raster shape fixed (two-launch step); per-launch raster
ms of: reset + 30 random-action steps, 30 more (no reset), reset + 30 again, reset + 30 steps of the
constant action 10."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flow_field_based_motion_planner_amd.vec_env import FFMPVec  # noqa: E402

dev = torch.device("cuda:0")
env = FFMPVec(32768, "C3", device=dev, tuning={"shape": [4096, 37], "shape_newest": [4096, 37], "fused": False,
                                                 "fused_flags": 37})
gen = torch.Generator(device=dev).manual_seed(1000)
acts = torch.randint(0, 28, (30, 32768), device=dev, dtype=torch.int64, generator=gen)
const = torch.full((30, 32768), 10, dtype=torch.int64, device=dev)


def run(tag, reset, a):
    torch.cuda.synchronize()
    if reset:
        env.reset()
    e0 = int(env.episode.sum())
    t = []
    for k in range(30):
        env.step(a[k], timing=t)
    torch.cuda.synchronize()
    ms = [r[0].elapsed_time(r[1]) for r in t]
    print(f"{tag:8s} resets {int(env.episode.sum()) - e0:6d} " + " ".join(f"{x:.2f}" for x in ms), flush=True)


run("reset", True, acts)
run("cont", False, acts)
run("reset2", True, acts)
run("const", True, const)
run("reset3", True, acts)
