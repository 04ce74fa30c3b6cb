"""FFMPVec.capture / StepGraph.replay: whole steps replayed from one HIP graph give the same states,
observations and flags as the same steps through step(), bit for bit, for each ring layout (seamless
W = 8 and W = 3, wrapping W = 4, contiguous W = 2) and for the one-launch step; the host's frame
bookkeeping (the state_m view) follows the replays."""
import numpy as np
import pytest
import torch

from flow_field_based_motion_planner_amd.config import FFMPConfig
from flow_field_based_motion_planner_amd.vec_env import FFMPVec

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
CFG = dict(grid=64, n_obst=8, n_beams=48, moving=True, obst_rmax=0.45, obst_vmax=1.0, world_half=2.4,
           goal_min=0.6, goal_max=1.5, max_steps=7, seed=31)


def _snap(env):
    d = {k: v.detach().cpu().numpy().copy() for k, v in env.obs.items()}
    for k in ("reward", "done", "is_goal", "collision", "truncated", "pose", "goal", "obst", "t", "episode", "record"):
        d[k] = getattr(env, k).detach().cpu().numpy().copy()
    return d


@pytest.mark.parametrize("window,seamless,fused", [(8, True, False), (3, True, False), (4, False, False),
                                                    (2, False, False), (8, True, True)])
def test_graph_replay_equals_steps(window, seamless, fused):
    cfg = FFMPConfig(**CFG)
    n = 96
    a = FFMPVec(n, cfg, device=DEV, frame_window=window, seamless=seamless if window > 2 else None, fused=fused,
                autotune=False)
    b = FFMPVec(n, cfg, device=DEV, frame_window=window, seamless=seamless if window > 2 else None, fused=fused,
                autotune=False)
    per = a.graph_period()
    assert per == (window if seamless else max(window - 1, 1))
    rng = np.random.default_rng(5)
    acts = torch.as_tensor(rng.integers(0, 28, (4 * per + 3, n)), device=DEV)
    a.reset()
    b.reset()
    for k in range(3):  # off the reset position: the capture starts mid-ring
        a.step(acts[k])
        b.step(acts[k])
    g = a.capture()
    with pytest.raises(ValueError):
        a.capture(0)
    for r in range(4):
        blk = acts[3 + r * per:3 + (r + 1) * per]
        g.replay(blk)
        for k in range(per):
            b.step(blk[k])
        torch.cuda.synchronize()
        sa, sb = _snap(a), _snap(b)
        for k in sb:
            assert np.array_equal(sa[k], sb[k], equal_nan=True), (r, k)
    assert int(a.done.sum()) >= 0 and int(b.episode.sum()) > 0  # resets happened inside the replays
    if per > 1:
        # a partial graph (fewer steps than the period) replays from the capture's position once
        part = a.capture(per - 1)
        assert not part.chainable
        blk = acts[:per - 1]
        part.replay(blk)
        for k in range(per - 1):
            b.step(blk[k])
        torch.cuda.synchronize()
        sa, sb = _snap(a), _snap(b)
        for k in sb:
            assert np.array_equal(sa[k], sb[k], equal_nan=True), ("partial", k)
        # the frame position moved: both graphs refuse until it is back where they were captured
        with pytest.raises(RuntimeError):
            g.replay()
        a.step(acts[0])
        b.step(acts[0])
        g.replay(acts[1:per + 1])
        for k in range(1, per + 1):
            b.step(acts[k])
        torch.cuda.synchronize()
        sa, sb = _snap(a), _snap(b)
        for k in sb:
            assert np.array_equal(sa[k], sb[k], equal_nan=True), ("after partial", k)
    a.close()
    b.close()
