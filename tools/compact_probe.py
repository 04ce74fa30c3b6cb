"""Where does the compact-format (uint8 frames, float16 potential) raster spend its time at C3?
Newest-only launches in the step loop (HIP events, two-launch step), autotuned shape per variant:
the C3 raster, without the potential plane (frames only), K = 0 (no disc work), the repulsive reach
cut to 0.05 m, and the float32 layout for comparison.
usage: python tools/compact_probe.py"""
import gc
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from flow_field_based_motion_planner_amd.config import preset  # noqa: E402
from flow_field_based_motion_planner_amd.vec_env import FFMPVec  # noqa: E402

N = 32768
variants = [("u8f16 C3", preset("C3"), {}), ("u8 frames only", preset("C3"), {"potential": False}),
            ("u8f16 K=0", preset("C3", n_obst=0), {}), ("u8f16 rho0=0.05", preset("C3", rho0=0.05), {}),
            ("u8f16 C3 again", preset("C3"), {})]
for name, cfg, kw in variants:
    env = FFMPVec(N, cfg, device="cuda:0", obs_format="u8f16", fused=False, **kw)
    env.reset()
    gen = torch.Generator(device="cuda:0").manual_seed(5)
    acts = torch.randint(0, 28, (24, N), device="cuda:0", generator=gen)
    for k in range(4):
        env.step(acts[k])
    t = []
    for k in range(4, 24):
        env.step(acts[k], timing=t)
    torch.cuda.synchronize()
    ms = [r[0].elapsed_time(r[1]) for r in t]
    b = sum(r[3] for r in t)
    print(f"{name:16s} shape {env.raster_shape_newest} ring {env.ring}: raster {sum(ms) / len(ms):.3f} ms, "
          f"{b / (sum(ms) * 1e-3) / 1e9:.0f} GB/s (resets excluded), tuned {env.placement['gbs']}", flush=True)
    print("   candidates (cells/block, flags, newest-only GB/s):",
          " ".join(f"{c[0]}/{c[1]}:{c[-1]:.0f}" for c in env.placement["candidates"]), flush=True)
    env.close()
    del env
    gc.collect()
