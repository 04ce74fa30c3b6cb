"""Several C3 FFMPVec instances in one process: autotune candidates (cycle-averaged newest-only
GB/s per launch shape), ring pairing info and per-slot raster ms of the chosen shape."""
import gc
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from flow_field_based_motion_planner_amd.config import preset  # noqa: E402
from flow_field_based_motion_planner_amd.vec_env import FFMPVec  # noqa: E402

for trial in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    env = FFMPVec(32768, preset("C3"), device="cuda:0")
    pl = env.placement
    print(f"trial {trial}: chosen {pl['shape_newest']} cycle {pl['gbs']} GB/s; ring {dict((k, v) for k, v in pl['ring'].items() if k != 'repair')}")
    print("   repair:", pl["ring"]["repair"])
    print("   candidates:", " ".join(f"{c[0]}/{c[1]}:{c[-1]:.0f}" for c in pl["candidates"]), flush=True)
    del env
    gc.collect()
