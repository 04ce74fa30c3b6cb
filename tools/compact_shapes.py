"""Compact-format (uint8 frames, float16 potential) newest-only raster at C3 for a list of launch
shapes, on ONE instance (no autotune): mean raster ms per launch over 2 x 8 steps of the real step
loop (HIP events around each raster launch).  Usage: python tools/compact_shapes.py [cfg] [f32|u8f16]
[blocks:flags,...] [reps] (default: the SHAPES list below, 2 reps)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from flow_field_based_motion_planner_amd import _abi  # noqa: E402
from flow_field_based_motion_planner_amd.config import PRESETS  # noqa: E402
from flow_field_based_motion_planner_amd.vec_env import FFMPVec  # noqa: E402

NT, PL, XCD = _abi.RASTER_NT, _abi.RASTER_PLAIN, _abi.RASTER_XCD
T2, T4, T8, T16, NAR = _abi.RASTER_TILE2, _abi.RASTER_TILE4, _abi.RASTER_TILE8, _abi.RASTER_TILE16, _abi.RASTER_NARROW
M8 = _abi.RASTER_MID8
SHAPES = [(65536, NT | T4 | NAR), (65536, NT | T2 | NAR),
          # round 3: 8 cells per lane (FFMP_RASTER_MID8)
          (65536, NT | T4 | M8), (32768, NT | T4 | M8), (65536, NT | XCD | T4 | M8), (65536, PL | T4 | M8),
          (16384, NT | T4 | M8), (65536, NT | T8 | M8)]


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "C3"
    fmt = sys.argv[2] if len(sys.argv) > 2 else "u8f16"
    shapes = SHAPES
    if len(sys.argv) > 3 and sys.argv[3]:
        shapes = [tuple(int(v) for v in t.split(":")) for t in sys.argv[3].split(",")]
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    pr = PRESETS[name]
    n = pr["n_envs"] // max(1, pr["gpus"])
    env = FFMPVec(n, name, device="cuda:0", obs_format=fmt, autotune=False, fused=False)
    a = torch.full((n,), 10, dtype=torch.int64, device="cuda:0")
    for rep in range(reps):
        for shape in shapes:
            env.raster_shape = env.raster_shape_newest = shape
            env.reset()
            for _ in range(2):
                env.step(a)
            t = []
            for _ in range(8):
                env.step(a, timing=t)
            torch.cuda.synchronize()
            ms = [r[0].elapsed_time(r[1]) for r in t]
            b = sum(r[3] for r in t)
            print(f"rep {rep} shape {shape[0]:6d}/{shape[1]:4d}: raster {sum(ms) / len(ms):.3f} ms "
                  f"{b / (sum(ms) * 1e-3) / 1e9:.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
