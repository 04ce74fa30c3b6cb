#!/usr/bin/env python3
"""Why bench.py's remainder replay (K % graph_period() steps) runs slower per step than the full-period
replays: C3, an 8-step graph and 4-step graphs captured at ring positions 0 and 4, timed with HIP
events in several orders (profiles/r06h_rem_probe.txt)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flow_field_based_motion_planner_amd.config import preset  # noqa: E402
from flow_field_based_motion_planner_amd.vec_env import FFMPVec  # noqa: E402

dev = torch.device("cuda:0")
n = 32768
env = FFMPVec(n, preset("C3"), device=dev)
gen = torch.Generator(device=dev).manual_seed(1)
A = torch.randint(0, 28, (64, n), device=dev, dtype=torch.int64, generator=gen)
env.reset()
for w in range(8):
    env.step(A[w])
g8 = env.capture()
g4a = env.capture(4)
for w in range(4):
    env.step(A[w])
g4b = env.capture(4)
for w in range(4):
    env.step(A[w])
torch.cuda.synchronize()


def t(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn()
    e1.record()
    return e0, e1


for _ in range(6):  # warm
    g8.replay(A[:8])
torch.cuda.synchronize()
for rnd in range(3):
    ev = []
    ev.append(("g8", t(lambda: g8.replay(A[:8]))))
    ev.append(("g8", t(lambda: g8.replay(A[8:16]))))
    ev.append(("g4a", t(lambda: g4a.replay(A[16:20]))))
    ev.append(("g4b", t(lambda: g4b.replay(A[20:24]))))
    ev.append(("g4a", t(lambda: g4a.replay(A[24:28]))))
    ev.append(("g4b", t(lambda: g4b.replay(A[28:32]))))
    ev.append(("g8", t(lambda: g8.replay(A[32:40]))))
    torch.cuda.synchronize()
    print(" | ".join(f"{k} {a.elapsed_time(b) / (8 if k == 'g8' else 4):.3f}" for k, (a, b) in ev), flush=True)
# step() one at a time for comparison
ev = []
for w in range(8):
    ev.append(t(lambda: env.step(A[w])))
torch.cuda.synchronize()
print("step() ms:", " ".join(f"{a.elapsed_time(b):.3f}" for a, b in ev), flush=True)
# the bench's timed sequence under ONE event pair (gaps between replays included) against the sum of
# per-replay events
for rnd in range(3):
    torch.cuda.synchronize()
    per = []
    L0, L1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    L0.record()
    per.append(t(lambda: g8.replay(A[:8])))
    per.append(t(lambda: g8.replay(A[8:16])))
    per.append(t(lambda: g4a.replay(A[16:20])))
    L1.record()
    torch.cuda.synchronize()
    s = sum(a.elapsed_time(b) for a, b in per)
    print(f"loop {L0.elapsed_time(L1):.3f} ms, replays {s:.3f} ms, gaps {L0.elapsed_time(L1) - s:.3f} ms", flush=True)
    for w in range(4):
        env.step(A[w])
    torch.cuda.synchronize()
# the same without per-replay events
import time  # noqa: E402
for rnd in range(3):
    torch.cuda.synchronize()
    L0, L1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    h0 = time.perf_counter()
    L0.record()
    g8.replay(A[:8])
    h1 = time.perf_counter()
    g8.replay(A[8:16])
    h2 = time.perf_counter()
    g4a.replay(A[16:20])
    h3 = time.perf_counter()
    L1.record()
    torch.cuda.synchronize()
    h4 = time.perf_counter()
    print(f"loop {L0.elapsed_time(L1):.3f} ms (20 steps: {L0.elapsed_time(L1) / 20:.4f}/step); host launch ms "
          f"{(h1 - h0) * 1e3:.3f} {(h2 - h1) * 1e3:.3f} {(h3 - h2) * 1e3:.3f}; wall {(h4 - h0) * 1e3:.3f}", flush=True)
    for w in range(4):
        env.step(A[w])
    torch.cuda.synchronize()
