"""Where a step's time goes inside the kernels: wall-clock stamps (100 MHz) from a probe build of
libffmp (-DFFMP_TRACE, tools/gpu_trace.sh) at checkpoints of the env step (per env) and of the
raster (per block).  Prints, for one two-launch step, the per-phase latency of the env step,
the dispatch skew of waves / blocks, and the raster's block timeline.
usage: FFMP_LIB=tools/_build/libffmp_trace.so python tools/trace_probe.py [preset] [n_envs]"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from flow_field_based_motion_planner_amd import _abi  # noqa: E402
from flow_field_based_motion_planner_amd.config import preset  # noqa: E402
from flow_field_based_motion_planner_amd.vec_env import FFMPVec  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C2"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
fused = len(sys.argv) > 3 and sys.argv[3] == "fused"
lib = _abi.load()
lib.ffmp_trace_read.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
env_t = np.zeros((4096, 12), np.uint64)
ras_t = np.zeros((65536, 4), np.uint64)

env = FFMPVec(n, preset(name), device="cuda:0", fused=fused)
env.reset()
acts = torch.randint(0, 28, (40, n), device="cuda:0")
for k in range(30):
    env.step(acts[k])
torch.cuda.synchronize()
lib.ffmp_trace_read(env_t.ctypes.data, ras_t.ctypes.data, 1)
print(f"{name} n={n} shape={env.raster_shape_newest if hasattr(env, 'raster_shape_newest') else '?'}", flush=True)
if fused:  # one block per env: env step (wave 0) then the block's raster; stamps 0 / 3 / 2
    for rep in range(3):
        env.step(acts[30 + rep])
        torch.cuda.synchronize()
        lib.ffmp_trace_read(env_t.ctypes.data, ras_t.ctypes.data, 1)
        R = ras_t[:min(n, 65536)].astype(np.int64)
        r0 = R[:, 0].min()
        us = lambda a: a * 0.01
        envp, rasp, tot = R[:, 3] - R[:, 0], R[:, 2] - R[:, 3], R[:, 2] - R[:, 0]
        print(f"-- fused step {rep}: span {us(R[:, 2].max() - r0):.1f} us, {len(R)} blocks")
        for nm, d in (("env phase", envp), ("raster phase", rasp), ("block", tot)):
            print(f"   {nm:14s} median {us(np.median(d)):7.2f}  p10 {us(np.percentile(d, 10)):7.2f}  "
                  f"p90 {us(np.percentile(d, 90)):7.2f}  max {us(d.max()):7.2f} us")
        print(f"   env-phase share of block time: {envp.sum() / tot.sum():.3f}")
        E = env_t[:min(n, 4096)].astype(np.int64)
        names = ["load+integrate", "lidar_disc+cos/sin+ego", "collide+lidar+reward", "reset", "grad+record",
                 "writes"]
        for k in range(6):
            d = E[:, k + 1] - E[:, k]
            print(f"   env {names[k]:24s} median {us(np.median(d)):6.2f}  p90 {us(np.percentile(d, 90)):6.2f} us")
        for a, b, nm in ((2, 7, "  footprint"), (7, 8, "  lidar scene + beams"), (8, 9, "  ballots, reward, state_g")):
            d = E[:, b] - E[:, a]
            print(f"   env {nm:24s} median {us(np.median(d)):6.2f}  p90 {us(np.percentile(d, 90)):6.2f} us")
    sys.exit(0)
for rep in range(3):
    env.step(acts[30 + rep])
    torch.cuda.synchronize()
    lib.ffmp_trace_read(env_t.ctypes.data, ras_t.ctypes.data, 1)
    ne = min(n, 4096)
    E = env_t[:ne].astype(np.int64)
    t0 = E[:, 0].min()
    us = lambda a: a * 0.01  # 100 MHz ticks -> us
    print(f"-- step {rep}: env kernel span {us(E[:, 6].max() - t0):.1f} us (first {ne} envs)")
    print(f"   wave start skew: median {us(np.median(E[:, 0] - t0)):.2f}  max {us((E[:, 0] - t0).max()):.2f} us")
    names = ["load+integrate", "lidar_disc+cos/sin+ego", "collide+lidar+reward", "reset", "grad+record",
             "writes"]
    for k in range(6):
        d = E[:, k + 1] - E[:, k]
        print(f"   {names[k]:24s} median {us(np.median(d)):6.2f}  p99 {us(np.percentile(d, 99)):6.2f}  "
              f"max {us(d.max()):6.2f} us")
    for a, b, nm in ((2, 7, "  footprint"), (7, 8, "  lidar scene + beams"), (8, 9, "  ballots, reward, state_g"),
                     (9, 3, "  terminal record")):
        d = E[:, b] - E[:, a]
        print(f"   {nm:24s} median {us(np.median(d)):6.2f}  p99 {us(np.percentile(d, 99)):6.2f}  "
              f"max {us(d.max()):6.2f} us")
    tot = E[:, 6] - E[:, 0]
    print(f"   {'per-env total':24s} median {us(np.median(tot)):6.2f}  max {us(tot.max()):6.2f} us")
    Rr = ras_t.astype(np.int64)
    used = Rr[:, 0] > 0
    if used.any():
        R = Rr[used]
        r0 = R[:, 0].min()
        print(f"   raster: {used.sum()} blocks traced; starts {us(r0 - E[:, 6].max()):.2f} us after the env kernel's "
              f"last stamp; span {us(R[:, 2].max() - r0):.1f} us")
        print(f"   raster block: record load median {us(np.median(R[:, 1] - R[:, 0])):.2f} us, "
              f"whole block median {us(np.median(R[:, 2] - R[:, 0])):.2f}  p99 {us(np.percentile(R[:, 2] - R[:, 0], 99)):.2f} us")
        st = np.sort(R[:, 0] - r0)
        en = np.sort(R[:, 2] - r0)
        for q in (0.01, 0.1, 0.5, 0.9, 0.99, 1.0):
            i = min(int(q * len(st)), len(st) - 1)
            print(f"     {q:5.2f} of blocks started by {us(st[i]):7.2f} us, ended by {us(en[i]):7.2f} us")
