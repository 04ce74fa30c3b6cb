"""C3 raster (fixed 4096-cell plain shape) launched 6 times after 3 steps; meant to run under
rocprofv3 --pmc so per-dispatch counters and timestamps come from ONE placement."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from flow_field_based_motion_planner_amd.config import preset  # noqa: E402
from flow_field_based_motion_planner_amd.vec_env import FFMPVec  # noqa: E402

shape = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (4096, 2)
env = FFMPVec(32768, preset("C3"), device="cuda:0", autotune=False)
env.raster_shape = shape
env.reset()
a = torch.full((32768,), 10, dtype=torch.int64, device="cuda:0")
for _ in range(3):
    env.step(a)
for _ in range(6):
    env.raster()
torch.cuda.synchronize()
