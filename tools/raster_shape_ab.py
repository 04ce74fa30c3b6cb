"""Raster launch shapes A/B on the SAME allocations (several fresh ones): cells per block x
XCD remap.  Usage: python tools/raster_shape_ab.py [preset] [allocs]"""
import gc
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from flow_field_based_motion_planner_amd import _abi  # noqa: E402
from flow_field_based_motion_planner_amd.config import PRESETS, bytes_per_env_step, preset  # noqa: E402
from flow_field_based_motion_planner_amd.vec_env import FFMPVec  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C3"
allocs = int(sys.argv[2]) if len(sys.argv) > 2 else 4
cfg = preset(name)
pr = PRESETS[name]
N = pr["n_envs"] // max(pr["gpus"], 1)
b = bytes_per_env_step(cfg)["raster"] * N
shapes = [(4096, 0), (4096, 1), (2048, 0), (2048, 1), (1024, 0), (1024, 1)]
print(name, "N", N, "GB/s per (cells/block, xcd):", shapes, flush=True)
for r in range(allocs):
    env = FFMPVec(N, cfg, device="cuda:0", autotune=False)
    env.reset()
    row = []
    for cpb, xcd in shapes:
        _abi.set_tuning(_abi.TUNE_RASTER_CPB, cpb)
        _abi.set_tuning(_abi.TUNE_RASTER_XCD, xcd)
        env.raster()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(6):
            env.raster()
        ev[1].record()
        torch.cuda.synchronize()
        row.append(b / (ev[0].elapsed_time(ev[1]) / 6) / 1e6)
    print(f"alloc {r}: " + " | ".join(f"{v:.0f}" for v in row), flush=True)
    del env
    gc.collect()
    torch.cuda.empty_cache()
