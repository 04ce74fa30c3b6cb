"""Raster GB/s for each shape on ONE instance under three regimes:
   A: back-to-back rasters right after reset (what the autotuner timed)
   B: back-to-back rasters after 5 env steps
   C: steady-state step loop (env kernel + raster), raster timed per launch."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from flow_field_based_motion_planner_amd.config import PRESETS, bytes_per_env_step, preset  # noqa: E402
from flow_field_based_motion_planner_amd.vec_env import FFMPVec  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C3"
cfg = preset(name)
pr = PRESETS[name]
N = pr["n_envs"] // max(pr["gpus"], 1)
b = bytes_per_env_step(cfg)["raster"] * N
env = FFMPVec(N, cfg, device="cuda:0", autotune=False)
acts = torch.randint(0, 28, (40, N), device="cuda:0")


def rasters(k=4):
    env.raster()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(k):
        env.raster()
    ev[1].record()
    torch.cuda.synchronize()
    return b / (ev[0].elapsed_time(ev[1]) / k) / 1e6


for shape in [(4096, 2), (2048, 2), (2048, 6), (2048, 1)]:
    env.raster_shape = shape
    env.reset()
    a = rasters()
    for k in range(5):
        env.step(acts[k])
    bb = rasters()
    t = []
    for k in range(5, 25):
        env.step(acts[k], timing=t)
    torch.cuda.synchronize()
    c = b / (sum(x.elapsed_time(y) for x, y, *_ in t) / len(t)) / 1e6
    print(f"{name} shape {shape}: A {a:.0f}  B {bb:.0f}  C {c:.0f}", flush=True)
