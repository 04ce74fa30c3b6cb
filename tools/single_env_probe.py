#!/usr/bin/env python3
"""Per-call latency of the drop-in single-env surface (env.FFMP) on the GPU box, beside the
reference's own CPU figures (BASELINE.md §1 / SURVEY §6: rewarder2 7.2 us at 180 beams, 14.8 us at
360; rewarder 2.54 ms at 100^2): FFMP.rewarder2 (the one env call src/train.py:577 makes per
step), FFMP.rewarder, FFMP.is_collision2, and the gym step() of a one-env FFMPVec.  Each call is a
host -> device copy of its packed inputs, one kernel and a device -> host copy (env.py)."""
import contextlib
import io
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flow_field_based_motion_planner_amd import env as envmod  # noqa: E402
from flow_field_based_motion_planner_amd.config import FFMPConfig  # noqa: E402


def per_call(fn, n=2000):
    for _ in range(50):
        fn()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    return (time.perf_counter() - t0) / n * 1e6


def main():
    rng = np.random.default_rng(0)
    e = envmod.FFMP(verbose=False)
    rg = np.array([3.0, 0.2])
    e.rewarder2([None] + [1.0] * 179, rg, True)
    rows = {}
    for L in (180, 360):
        scan = [None] + [float(v) for v in rng.uniform(0.2, 5.0, L - 1).astype(np.float32)]  # train.py:97,145-150
        rows[f"rewarder2 ({L} beams)"] = per_call(lambda: e.rewarder2(scan, rg, False))
        rows[f"is_collision2 ({L} beams)"] = per_call(lambda: e.is_collision2(scan))
    m = np.zeros((100, 100, 1), dtype=np.int32)
    m[rng.integers(0, 100, 300), rng.integers(0, 100, 300), 0] = 255
    m[45:56, 45:56] = 0
    rows["rewarder (100x100 map)"] = per_call(lambda: e.rewarder(m, rg, False), 1000)
    rows["is_collision (100x100 map)"] = per_call(lambda: e.is_collision(m), 1000)
    g = envmod.FFMP(FFMPConfig(grid=100, n_obst=4, n_beams=180, autoreset=False, seed=3), verbose=False)
    g.reset()

    def step():
        with contextlib.redirect_stdout(io.StringIO()):
            _, _, done, _ = g.step(int(rng.integers(0, 28)))
        if done:
            g.reset()
    rows["gym step (1 env, 100x100, 180 beams; obs + info to host)"] = per_call(step, 300)
    ref = {"rewarder2 (180 beams)": 7.2, "rewarder2 (360 beams)": 14.8, "rewarder (100x100 map)": 2540.0}
    for k, us in rows.items():
        r = ref.get(k)
        print(f"{k:60s} {us:9.1f} us" + (f"   (reference CPU {r} us: {us / r:.2f}x)" if r else ""), flush=True)


if __name__ == "__main__":
    main()
