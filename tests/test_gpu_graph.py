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


@pytest.mark.parametrize("window,seamless", [(8, True), (3, True), (4, False), (2, False)])
def test_pipelined_graph_equals_steps(window, seamless):
    """The pipelined graph (env kernel of step i + 1 beside the raster of step i, two record
    buffers) against plain step() calls: same states, frames, potential and record after every
    replay, bit for bit; odd step counts and the one-launch step refuse it."""
    cfg = FFMPConfig(**CFG)
    n = 96
    kw = dict(device=DEV, frame_window=window, seamless=seamless if window > 2 else None, autotune=False)
    a = FFMPVec(n, cfg, fused=False, **kw)
    b = FFMPVec(n, cfg, fused=False, **kw)
    per = a.graph_period()
    k = per if per % 2 == 0 else 2 * per
    rng = np.random.default_rng(9)
    acts = torch.as_tensor(rng.integers(0, 28, (5 * k, n)), device=DEV)
    a.reset()
    b.reset()
    for i in range(2):
        a.step(acts[i])
        b.step(acts[i])
    g = a.capture(k, pipelined=True)
    assert g.pipelined and g.chainable
    if k % 2 == 0 and k > 1:
        with pytest.raises(ValueError):
            a.capture(k - 1, pipelined=True)
    for r in range(4):
        blk = acts[2 + r * k:2 + (r + 1) * k]
        g.replay(blk)
        for i in range(k):
            b.step(blk[i])
        torch.cuda.synchronize()
        sa, sb = _snap(a), _snap(b)
        for key in sb:
            assert np.array_equal(sa[key], sb[key], equal_nan=True), (r, key)
    assert int(b.episode.sum()) > 0  # resets happened inside the replays
    # step() after replays keeps working on the same (current) record buffer
    a.step(acts[0])
    b.step(acts[0])
    torch.cuda.synchronize()
    sa, sb = _snap(a), _snap(b)
    for key in sb:
        assert np.array_equal(sa[key], sb[key], equal_nan=True), ("step after", key)
    assert a.hbm_bytes() > b.hbm_bytes()  # the second record buffer is accounted
    a.close()
    b.close()
    if window == 8:
        f = FFMPVec(n, cfg, fused=True, **kw)
        f.reset()
        with pytest.raises(ValueError):
            f.capture(k, pipelined=True)
        f.close()


@pytest.mark.parametrize("window,seamless,n_obst", [(8, True, 8), (8, True, 12), (3, True, 8), (4, False, 8),
                                                    (2, False, 8), (8, True, 0)])
def test_skewed_graph_equals_steps(window, seamless, n_obst):
    """The skewed graph (ONE launch per step: raster of step i + env step of step i + 1,
    ffmp_step_skewed, two record buffers) against plain step() calls: states, frames, potential,
    record and the last step's small outputs bit for bit after every replay, for each ring layout,
    8 and 16 lanes per env and no discs; the compact layout and odd counts refuse it."""
    cfg = FFMPConfig(**dict(CFG, n_obst=n_obst))
    n = 96
    kw = dict(device=DEV, frame_window=window, seamless=seamless if window > 2 else None, autotune=False)
    a = FFMPVec(n, cfg, fused=False, **kw)
    b = FFMPVec(n, cfg, fused=False, **kw)
    per = a.graph_period()
    k = per if per % 2 == 0 else 2 * per
    rng = np.random.default_rng(13)
    acts = torch.as_tensor(rng.integers(0, 28, (3 + 5 * k, n)), device=DEV)
    a.reset()
    b.reset()
    for i in range(3):
        a.step(acts[i])
        b.step(acts[i])
    g = a.capture(k, skewed=True)
    assert g.skewed and not g.pipelined and g.chainable
    with pytest.raises(ValueError):
        a.capture(k, skewed=True, pipelined=True)
    for r in range(4):
        blk = acts[3 + r * k:3 + (r + 1) * k]
        g.replay(blk)
        for i in range(k):
            b.step(blk[i])
        torch.cuda.synchronize()
        sa, sb = _snap(a), _snap(b)
        for key in sb:
            assert np.array_equal(sa[key], sb[key], equal_nan=True), (r, key)
    assert int(b.episode.sum()) > 0  # resets happened inside the replays
    a.step(acts[0])
    b.step(acts[0])
    torch.cuda.synchronize()
    sa, sb = _snap(a), _snap(b)
    for key in sb:
        assert np.array_equal(sa[key], sb[key], equal_nan=True), ("step after", key)
    a.close()
    b.close()
    if window == 8 and n_obst == 8:
        c = FFMPVec(n, cfg, fused=False, obs_format="u8f16", **kw)
        c.reset()
        assert not c.capture(k).skewed  # the default falls back to the two launches
        with pytest.raises(ValueError):
            c.capture(k, skewed=True)
        c.close()
