"""Time the env kernel alone (ffmp_step_state) for a preset; FFMP_ENV_WAVES selects the block shape."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from flow_field_based_motion_planner_amd.config import preset  # noqa: E402
from flow_field_based_motion_planner_amd.vec_env import FFMPVec  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C3"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 32768
env = FFMPVec(n, preset(name), device="cuda:0", autotune=False)
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
print(f"{name} n={n} env_waves={os.environ.get('FFMP_ENV_WAVES', '1')}: env kernel {ev[0].elapsed_time(ev[1]) / 50 * 1000:.1f} us")
