"""Host overhead of FFMPVec.step for small batches (launch-bound regime): wall time per step
vs GPU time per step (one event pair around the loop), for a few sizes.
usage: python tools/step_overhead.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from flow_field_based_motion_planner_amd import FFMPConfig  # noqa: E402
from flow_field_based_motion_planner_amd.vec_env import FFMPVec  # noqa: E402

for G, n, K, L in ((32, 64, 4, 0), (100, 256, 4, 180), (100, 4096, 4, 180), (64, 1024, 4, 0)):
    cfg = FFMPConfig(grid=G, n_obst=K, n_beams=L, moving=False, seed=1)
    for fused in (False, True):
        env = FFMPVec(n, cfg, device="cuda:0", fused=fused)
        env.reset()
        acts = torch.randint(0, 28, (600, n), device="cuda:0")
        for k in range(100):
            env.step(acts[k])
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        for k in range(100, 600):
            env.step(acts[k])
        e1.record()
        t_host = (time.perf_counter() - t0) / 500 * 1e6
        torch.cuda.synchronize()
        t_all = (time.perf_counter() - t0) / 500 * 1e6
        print(f"G={G:4d} n={n:5d} fused={fused!s:5s}: host enqueue {t_host:6.1f} us/step, wall {t_all:6.1f} us/step, "
              f"gpu span {e0.elapsed_time(e1) / 500 * 1e3:6.1f} us/step", flush=True)
        env.close()
