#!/usr/bin/env python3
"""bench.py's graph sequence replicated (warm-up of 5 steps, the 8-step graph and the skewed trial graph, the
4-step remainder graph captured at the same position), then the remainder replay timed against 4-step graphs
captured at other positions and at the same position after re-capture (profiles/r06h_rem_probe.txt)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flow_field_based_motion_planner_amd.config import preset  # noqa: E402
from flow_field_based_motion_planner_amd.vec_env import FFMPVec  # noqa: E402

dev = torch.device("cuda:0")
n = 32768
W = 5
env = FFMPVec(n, preset("C3"), device=dev)
gen = torch.Generator(device=dev).manual_seed(1)
A = torch.randint(0, 28, (64, n), device=dev, dtype=torch.int64, generator=gen)
int(env.episode.sum())
env.reset()
for w in range(W):
    env.step(A[w])
print("pos after warm-up", env._wpos, flush=True)
g8 = env.capture()
gs = env.capture(skewed=True)
for g in (g8, gs):
    g.replay(A[:8])
for _ in range(8):
    g8.replay(A[:8])
    gs.replay(A[:8])
g8.replay(A[:8])
g4 = env.capture(4)
g4.replay(A[:4])
for k in range(4, 8):
    env.step(A[k])
for _ in range(4):
    g8.replay(A[:8])
torch.cuda.synchronize()


def t(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn()
    e1.record()
    return e0, e1


def seq(g4x, label):
    for rnd in range(3):
        ev = [t(lambda: g8.replay(A[8:16])), t(lambda: g8.replay(A[16:24])), t(lambda: g4x.replay(A[24:28]))]
        for k in range(4, 8):
            env.step(A[k])
        torch.cuda.synchronize()
        print(label, " ".join(f"{a.elapsed_time(b) / (8 if i < 2 else 4):.3f}" for i, (a, b) in enumerate(ev)), flush=True)


seq(g4, "bench-order g4")
g4n = env.capture(4)  # recaptured at the same position
seq(g4n, "recaptured g4")
# one step at a time over a ring cycle: per-step ms by position
ev = []
for w in range(8):
    ev.append(t(lambda: env.step(A[w])))
torch.cuda.synchronize()
print("step() ms from pos", env._wpos, ":", " ".join(f"{a.elapsed_time(b):.3f}" for a, b in ev), flush=True)
# the 4-step graph's steps one by one: its env kernels and rasters under per-kernel events
for k in range(4):
    e = [t(lambda: env.step_state(A[k])), t(lambda: env.raster_step())]
    torch.cuda.synchronize()
    print("plain step", k, "env", f"{e[0][0].elapsed_time(e[0][1]):.3f}", "raster", f"{e[1][0].elapsed_time(e[1][1]):.3f}", flush=True)
