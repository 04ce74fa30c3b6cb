"""Where the env kernel's time goes, per phase, from a probe build with wall-clock stamps
(-DFFMP_TRACE: `make probe V=trace DEFS=-DFFMP_TRACE`; never the shipped library).  Stamps (100 MHz,
each after an s_waitcnt(0), lane 0 of every env group, first 4,096 envs) of env_group's checkpoints:
0 start, 1 integrated, 2 ego discs, 3 gradient + record + state written, 7 footprint, 8 lidar,
9 reward, 4 before the reset, 6 end.
usage: FFMP_LIB=tools/_probe/libffmp_trace.so python tools/env_trace_probe.py [preset] [n_envs]"""
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
lib = _abi.load()
lib.ffmp_trace_read.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
env_t = np.zeros((4096, 12), np.uint64)
ras_t = np.zeros((65536, 4), np.uint64)
env = FFMPVec(n, preset(name), device="cuda:0", fused=False, autotune=False)
env.reset()
acts = torch.randint(0, 28, (60, n), device="cuda:0")
for k in range(40):
    env.step(acts[k])
torch.cuda.synchronize()
PH = [(0, 1, "load + integrate"), (1, 2, "ego discs (cos/sin)"), (2, 3, "grad + record + state"),
      (3, 7, "footprint"), (7, 8, "lidar"), (8, 9, "reward + outputs"), (4, 6, "reset (all envs)")]
acc = {p[2]: [] for p in PH}
span, skew, tot = [], [], []
for rep in range(8):
    env.step(acts[40 + rep])
    torch.cuda.synchronize()
    lib.ffmp_trace_read(env_t.ctypes.data, ras_t.ctypes.data, 1)
    ne = min(n, 4096)
    E = env_t[:ne].astype(np.int64)
    t0 = E[:, 0].min()
    span.append((E[:, 6].max() - t0) * 0.01)
    skew.append(np.median(E[:, 0] - t0) * 0.01)
    tot.append(np.median(E[:, 6] - E[:, 0]) * 0.01)
    for a, b, nm in PH:
        acc[nm].append(E[:, b] - E[:, a])
print(f"{name} n={n}: stamped span (first {min(n, 4096)} envs) median {np.median(span):.2f} us, "
      f"group start skew median {np.median(skew):.2f} us, per-group chain median {np.median(tot):.2f} us")
for nm, v in acc.items():
    d = np.concatenate(v) * 0.01
    print(f"   {nm:24s} median {np.median(d):6.2f}  p90 {np.percentile(d, 90):6.2f}  max {d.max():6.2f} us  "
          f"(nonzero {np.mean(d > 0.05):.3f})")
