#!/usr/bin/env python3
"""Raster GB/s of the frame-window launch kinds (newest-only vs full) per launch shape, C3.
Usage: python tools/window_probe.py [W]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flow_field_based_motion_planner_amd import _abi, preset  # noqa: E402
from flow_field_based_motion_planner_amd.vec_env import FFMPVec  # noqa: E402

W = int(sys.argv[1]) if len(sys.argv) > 1 else 8
env = FFMPVec(32768, preset("C3"), device="cuda:0", frame_window=W, autotune=False)
env.reset()
a = torch.full((env.num_envs,), 10, dtype=torch.int64, device="cuda:0")
shapes = [(c, f) for c in (2048, 4096, 8192, 16384) for f in (_abi.RASTER_NT, _abi.RASTER_PLAIN)]
shapes += [(c, f | _abi.RASTER_XCD) for c in (4096, 8192) for f in (_abi.RASTER_NT, _abi.RASTER_PLAIN)]
for rep in range(2):
    for shape in shapes:
        env.raster_shape = shape
        for _ in range(W - 1):
            env.step(a)
        t = []
        for _ in range(2 * (W - 1)):
            env.step(a, timing=t)
        torch.cuda.synchronize()
        out = {}
        for full in (True, False):
            sel = [r for r in t if r[4] == full]
            ms = sum(r[0].elapsed_time(r[1]) for r in sel)
            b = sum(r[3] for r in sel)
            out["full" if full else "newest"] = (b / (ms * 1e-3) / 1e9, ms / len(sel))
        tot_ms = sum(r[0].elapsed_time(r[1]) for r in t) / len(t)
        print(f"rep {rep} cpb {shape[0]:5d} flags {shape[1]:2d}: newest {out['newest'][0]:7.1f} GB/s "
              f"({out['newest'][1]:.3f} ms)  full {out['full'][0]:7.1f} GB/s ({out['full'][1]:.3f} ms)  "
              f"mean {tot_ms:.3f} ms/launch", flush=True)
