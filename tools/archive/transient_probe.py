#!/usr/bin/env python3
"""Where does the slow start of bench.py's timed loop come from?  One C3 FFMPVec (autotuned as in
bench.py), then per-launch raster times of 40 steps after reset() under three preludes:
  plain   reset, then the steps (bench.py with --warmup 0)
  idle    0.5 s of host sleep (GPU idle) before reset
  again   40 more steps right after the previous 40, no reset
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flow_field_based_motion_planner_amd.vec_env import FFMPVec  # noqa: E402

dev = torch.device("cuda:0")
gen = torch.Generator(device=dev).manual_seed(1000)
acts = torch.randint(0, 28, (40, 32768), device=dev, dtype=torch.int64, generator=gen)
env = FFMPVec(32768, "C3", device=dev, fused=(os.environ.get("FUSED", "auto") == "on") if os.environ.get("FUSED", "auto") != "auto" else None)
print("fused", env.fused, "shape", env.raster_shape_newest, flush=True)


def run(tag, reset=True, sleep=0.0):
    torch.cuda.synchronize()
    if sleep:
        time.sleep(sleep)
    if reset:
        env.reset()
    t = []
    for k in range(40):
        env.step(acts[k], timing=t)
    torch.cuda.synchronize()
    ms = [r[0].elapsed_time(r[1]) for r in t]
    print(f"{tag:6s} " + " ".join(f"{x:.2f}" for x in ms), flush=True)


run("plain")
run("again", reset=False)
run("idle", sleep=0.5)
run("again", reset=False)
run("plain")
run("idle2", sleep=2.0)
