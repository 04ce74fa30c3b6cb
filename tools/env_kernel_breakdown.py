"""Where the env kernel's time goes: time ffmp_step_state alone for variants of a preset (no lidar,
no obstacles, static obstacles, footprint-only collisions, fewer beams, no resets).
usage: python tools/env_kernel_breakdown.py [--preset C3] [--envs 32768] [variant ...]"""
import gc
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from flow_field_based_motion_planner_amd.config import preset  # noqa: E402
from flow_field_based_motion_planner_amd.vec_env import FFMPVec  # noqa: E402

args = sys.argv[1:]
base, n = "C3", 32768
while args and args[0].startswith("--"):
    if args[0] == "--preset":
        base = args[1]
    elif args[0] == "--envs":
        n = int(args[1])
    args = args[2:]
variants = {
    "base": {},
    "L=0 (no lidar)": dict(n_beams=0),
    "L=64": dict(n_beams=64),
    "K=0": dict(n_obst=0),
    "K=0,L=0": dict(n_obst=0, n_beams=0),
    "K=0,L=0,no collide": dict(n_obst=0, n_beams=0, collide_mode=0),
    "K=4": dict(n_obst=4),
    "static": dict(moving=False),
    "footprint only": dict(collide_mode=1),
    "lidar only": dict(collide_mode=2),
    "G=64 (same K, L)": dict(grid=64),
    "no resets": dict(collide_mode=0, max_steps=0, goal_thr=0.0),
}
only = args  # optional variant names to run
for name, kw in variants.items():
    if only and name not in only:
        continue
    env = FFMPVec(n, preset(base, **kw), device="cuda:0", autotune=False, frame_window=2, potential=False)
    env.reset()
    acts = torch.randint(0, 28, (60, n), device="cuda:0")
    for k in range(10):
        env.step_state(acts[k])
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    torch.cuda.synchronize()
    ev[0].record()
    for k in range(10, 60):
        env.step_state(acts[k])
    ev[1].record()
    torch.cuda.synchronize()
    print(f"{base} n={n} {name:20s}: env kernel {ev[0].elapsed_time(ev[1]) / 50 * 1000:7.1f} us", flush=True)
    del env
    gc.collect()
    torch.cuda.empty_cache()
