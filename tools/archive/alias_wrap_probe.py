"""Does slot 0 of the seamless ring run slow because the wrap step writes it through the alias
(virtual slot W)?  One C3 instance (autotune + repair as bench.py builds it), then the per-slot
newest-only raster times (FFMPVec._slot_ms, two ring cycles each) alternately with the wrap step
writing slot 0 through virtual slot W (WRAP_VIA_ALIAS True, the round-1 behaviour) and through
slot 0's own addresses (False, a negative frame stride).  Usage: python tools/alias_wrap_probe.py [C3] [reps]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from flow_field_based_motion_planner_amd.vec_env import FFMPVec  # noqa: E402
from flow_field_based_motion_planner_amd.config import PRESETS  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    pr = PRESETS[cfg]
    n = pr["n_envs"] // max(1, pr["gpus"])
    env = FFMPVec(n, cfg, device="cuda:0")
    print(json.dumps({"ring": env.ring_meta, "tuning": env.tuning()}), flush=True)
    for r in range(reps):
        for via_alias in (True, False):
            env.WRAP_VIA_ALIAS = via_alias
            ms = env._slot_ms()
            print(json.dumps({"rep": r, "via_alias": via_alias, "slot_ms": [round(ms[i], 3) for i in sorted(ms)],
                              "mean": round(sum(ms.values()) / len(ms), 4)}), flush=True)
    for via_alias in (True, False):
        env.WRAP_VIA_ALIAS = via_alias
        print(json.dumps({"sweep_via_alias": via_alias, "slot_ms": slot_sweep(env)}), flush=True)
    torch.cuda.synchronize()




def slot_sweep(env, order=(3, 0, 5, 1, 7, 2, 6, 4), reps=3):
    """Raster-only (no env kernel, fixed record) newest-only launches aimed at each physical slot
    in a shuffled order: if slot 0 is still slow out of the step sequence, it is the memory."""
    W = env.frame_window
    env.reset()
    a = torch.full((env.num_envs,), 10, dtype=torch.int64, device=env.device)
    env.step(a)
    out = {}
    for _ in range(reps):
        for s in order:
            if s >= W:
                continue
            env._set_window((s - 1) % W)  # newest at virtual s (s = 0: virtual W or slot 0 itself)
            t = []
            env._raster_launch(False, None, t)
            torch.cuda.synchronize()
            out.setdefault(s, []).append(t[0][0].elapsed_time(t[0][1]))
    env._clear_after_tuning()
    return {s: [round(x, 3) for x in v] for s, v in sorted(out.items())}


if __name__ == "__main__":
    main()
