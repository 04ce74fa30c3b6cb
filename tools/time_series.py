"""Raster store bandwidth over time on ONE fixed allocation (is the fast/slow mode time-dependent?)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from flow_field_based_motion_planner_amd.config import bytes_per_env_step, preset  # noqa: E402
from flow_field_based_motion_planner_amd.vec_env import FFMPVec  # noqa: E402

cfg = preset("C3")
N = 32768
env = FFMPVec(N, cfg, device="cuda:0", autotune=False)
env.reset()
b = bytes_per_env_step(cfg)["raster"] * N
t0 = time.time()
gap = float(sys.argv[1]) if len(sys.argv) > 1 else 0.0
for k in range(int(sys.argv[2]) if len(sys.argv) > 2 else 120):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(5):
        env.raster()
    ev[1].record()
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / 5
    print(f"{time.time() - t0:7.3f} {b / ms / 1e6:6.0f}", flush=True)
    if gap:
        time.sleep(gap)
