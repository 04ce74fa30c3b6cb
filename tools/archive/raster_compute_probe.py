"""Is the newest-only raster store-bound or compute-bound at C3?  Same shape (32,768 envs,
256^2, seamless ring; the pooled ring and the cached arena give every variant the same
memory), disc work varied: K = 16 (C3), K = 0 (attractive potential only), K = 16 with the
repulsive reach cut to 0.05 m (fewer discs survive the cull).  Raster GB/s of newest-only
launches in the step loop (HIP events), autotuned shape per variant.
usage: python tools/raster_compute_probe.py"""
import gc
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from flow_field_based_motion_planner_amd.config import preset  # noqa: E402
from flow_field_based_motion_planner_amd.vec_env import FFMPVec  # noqa: E402

N = 32768
variants = [("C3 K=16", preset("C3")), ("K=0", preset("C3", n_obst=0)), ("K=16 rho0=0.05", preset("C3", rho0=0.05)),
            ("C3 K=16 again", preset("C3"))]
if len(sys.argv) > 1 and sys.argv[1] == "C3only":
    variants = [("C3 K=16", preset("C3")), ("C3 K=16 again", preset("C3")), ("C3 K=16 third", preset("C3"))]
for name, cfg in variants:
    env = FFMPVec(N, cfg, device="cuda:0")
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
    del env
    gc.collect()
