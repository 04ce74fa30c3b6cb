"""Closed-loop stepping: the reference loop picks each action from the previous
observation (src/train.py:572-577) and publishes it (:665-682), so actions are never known a step
ahead.  Covered here:

* FFMPVec.use_graphs(True): step() as single-step HIP graph replays (one per frame-ring position) ==
  plain step() launches, bit for bit, over two ring cycles with auto-resets, a full reset and a
  reseed in between, for each ring layout, the one-launch step and the compact layout;
* FFMPVec.policy_reactive (include/ffmp.h ffmp_policy_reactive) == its NumPy restatement;
* capture(policy="reactive") (the policy inside the graph) == a loop of step(policy_reactive());
* StepGraph.skew_supported asks the library (ffmp_step_skewed_check), ADVICE r05;
* info_format="list": gym 0.17/0.18 VectorEnv's per-env info dicts."""
import ctypes as C

import numpy as np
import pytest
import torch

from flow_field_based_motion_planner_amd import _abi
from flow_field_based_motion_planner_amd.config import FFMPConfig
from flow_field_based_motion_planner_amd.vec_env import FFMPVec, StepGraph

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
CFG = dict(grid=64, n_obst=8, n_beams=48, moving=True, obst_rmax=0.45, obst_vmax=1.0, world_half=2.4,
           goal_min=0.6, goal_max=1.5, max_steps=7, seed=31)


def _snap(env):
    d = {k: v.detach().cpu().numpy().copy() for k, v in env.obs.items()}
    for k in ("reward", "done", "is_goal", "collision", "truncated", "pose", "goal", "obst", "t", "episode", "record"):
        d[k] = getattr(env, k).detach().cpu().numpy().copy()
    return d


def _same(a, b, where):
    sa, sb = _snap(a), _snap(b)
    for k in sb:
        assert np.array_equal(sa[k], sb[k], equal_nan=True), (where, k)


@pytest.mark.parametrize("window,seamless,fused,fmt", [(8, True, False, "f32"), (3, True, False, "f32"),
                                                        (4, False, False, "f32"), (2, False, False, "f32"),
                                                        (8, True, True, "f32"), (8, True, False, "u8f16")])
def test_step_graphs_equal_plain_steps(window, seamless, fused, fmt):
    cfg = FFMPConfig(**CFG)
    n = 96
    kw = dict(device=DEV, frame_window=window, seamless=seamless if window > 2 else None, fused=fused,
              autotune=False, obs_format=fmt)
    a, b = FFMPVec(n, cfg, **kw), FFMPVec(n, cfg, **kw)
    a.use_graphs(True)
    per = a.graph_period()
    rng = np.random.default_rng(7)
    acts = torch.as_tensor(rng.integers(0, 28, (2 * per + 9, n)), device=DEV)
    a.reset()
    b.reset()
    for k in range(2 * per + 3):  # two ring cycles, auto-resets inside (max_steps 7)
        a.step(acts[k])
        b.step(acts[k])
        _same(a, b, k)
    assert int(b.episode.sum()) > 0
    assert len(a._graphs) == per  # one graph per ring position
    # a full reset puts the ring back at slot 0: the same graphs keep serving
    a.reset()
    b.reset()
    for k in range(3):
        a.step(acts[2 * per + 3 + k])
        b.step(acts[2 * per + 3 + k])
        _same(a, b, ("after reset", k))
    # a reseed rebuilds the config the graphs captured by value: they are dropped and re-captured
    a.reset(seed=99)
    b.reset(seed=99)
    assert len(a._graphs) == 0
    for k in range(3):
        a.step(acts[2 * per + 6 + k])
        b.step(acts[2 * per + 6 + k])
        _same(a, b, ("after reseed", k))
    # the static action buffer itself: no copy
    a.action_buffer.copy_(acts[0])
    a.step(a.action_buffer)
    b.step(acts[0])
    _same(a, b, "action_buffer")
    a.use_graphs(False)
    a.step(acts[1])
    b.step(acts[1])
    _same(a, b, "graphs off")
    a.close()
    b.close()


def _policy_np(cfg, newest, state_g):
    """ffmp_policy_reactive restated (include/ffmp.h): newest (N, G, G), state_g (N, 2) float32."""
    G = cfg.grid
    look0, look1 = 3, min(3 + int(round(0.25 / cfg.res)), G // 2 - 1)
    orient = state_g[:, 1].astype(np.float32)
    wi = np.clip(np.rint(orient / np.float32(0.2)).astype(np.int64) + 3, 0, 6)
    ray = newest[:, G // 2 + look0:G // 2 + look1 + 1, G // 2]
    blocked = (ray > 0).any(1)
    vi = np.where(state_g[:, 0] < np.float32(1.0), 1, 3)
    vi = np.where(blocked, 0, vi)
    wi = np.where(blocked & (wi == 3), 6, wi)
    return 7 * vi + wi


@pytest.mark.parametrize("fmt", ["f32", "u8f16"])
def test_policy_reactive_matches_restatement(fmt):
    cfg = FFMPConfig(**dict(CFG, n_obst=16, obst_rmax=0.6, max_steps=40))
    n = 512
    env = FFMPVec(n, cfg, device=DEV, frame_window=4, autotune=False, obs_format=fmt)
    env.reset()
    rng = np.random.default_rng(3)
    seen_blocked = 0
    for k in range(12):
        a = env.policy_reactive()
        newest = env.state_m[:, 1].float().cpu().numpy()
        exp = _policy_np(cfg, newest, env.state_g.cpu().numpy())
        assert np.array_equal(a.cpu().numpy(), exp), k
        seen_blocked += int((a.cpu().numpy() // 7 == 0).sum())
        if k % 3 == 2:  # mix in random actions so robots end up facing discs
            a = torch.as_tensor(rng.integers(0, 28, n), device=DEV)
        env.step(a)
    assert seen_blocked > 0  # the look-ahead branch was exercised
    out = torch.empty(n, dtype=torch.int64, device=DEV)
    assert env.policy_reactive(out=out) is out
    with pytest.raises(ValueError):
        env.policy_reactive(out=torch.empty(n, dtype=torch.int32, device=DEV))
    env.close()


@pytest.mark.parametrize("window,seamless,fused", [(8, True, False), (4, False, False), (2, False, False),
                                                    (8, True, True)])
def test_closed_loop_graph_equals_step_loop(window, seamless, fused):
    cfg = FFMPConfig(**CFG)
    n = 96
    kw = dict(device=DEV, frame_window=window, seamless=seamless if window > 2 else None, fused=fused,
              autotune=False)
    a, b = FFMPVec(n, cfg, **kw), FFMPVec(n, cfg, **kw)
    a.reset()
    b.reset()
    for k in range(2):
        a.step(a.policy_reactive())
        b.step(b.policy_reactive())
    per = a.graph_period()
    g = a.capture(per * -(-8 // per), policy="reactive")  # >= 8 steps: truncations (max_steps 7) inside
    assert g.policy == "reactive" and not g.skewed and not g.pipelined and g.chainable
    with pytest.raises(ValueError):
        g.replay(torch.zeros((g.steps, n), dtype=torch.int64, device=DEV))
    with pytest.raises(ValueError):
        a.capture(policy="reactive", skewed=True)
    for r in range(3):
        g.replay()
        for k in range(g.steps):
            b.step(b.policy_reactive())
        torch.cuda.synchronize()
        _same(a, b, r)
    assert int(b.episode.sum()) > 0
    # a callable policy (torch ops, captured too): the greedy heading term only
    def heading(env):
        return (torch.clamp(torch.round(env.state_g[:, 1] / 0.2).to(torch.int64) + 3, 0, 6) + 14)
    g2 = a.capture(policy=heading)
    g2.replay()
    for k in range(g2.steps):
        b.step(heading(b))
    torch.cuda.synchronize()
    _same(a, b, "callable")
    a.close()
    b.close()


def test_skew_check_is_the_library_s():
    lib = _abi.load()
    cfg = FFMPConfig(**CFG)
    env = FFMPVec(64, cfg, device=DEV, frame_window=4, autotune=False)
    env.reset()
    assert lib.ffmp_step_skewed_check(C.byref(env._cfg_c), _abi.OBS_F32, 0) == 0
    assert StepGraph.skew_supported(env, 4)
    assert lib.ffmp_step_skewed_check(C.byref(env._cfg_c), _abi.OBS_U8F16, 0) == -1
    big = _abi.make_cfg(cfg.replace(n_beams=1024, n_obst=4), env.beam_cs.data_ptr())
    # 8 envs per wave x 4 waves x 1024 beams x 4 B = 128 KiB of keys + the static arrays: fits
    # only where a block may hold ~150 KiB of LDS; either way the answer is the library's own
    rc = lib.ffmp_step_skewed_check(C.byref(big), _abi.OBS_F32, 0)
    assert rc in (0, -1)
    if rc:
        assert b"LDS" in lib.ffmp_last_error()
    env.close()


def test_info_list_format():
    cfg = FFMPConfig(**CFG)
    n = 32
    a = FFMPVec(n, cfg, device=DEV, autotune=False, info_format="list")
    b = FFMPVec(n, cfg, device=DEV, autotune=False)
    with pytest.raises(ValueError):
        FFMPVec(n, cfg, device=DEV, autotune=False, info_format="tuple")
    a.reset()
    b.reset()
    rng = np.random.default_rng(1)
    for k in range(10):
        act = torch.as_tensor(rng.integers(0, 28, n), device=DEV)
        _, ra, da, ia = a.step(act)
        _, rb, db, ib = b.step(act)
        assert isinstance(ia, tuple) and len(ia) == n and all(isinstance(x, dict) for x in ia)
        for e in range(n):
            assert ia[e] == {key: (bool(ib[key][e]) if ib[key].dtype == torch.bool else int(ib[key][e]))
                             for key in ("is_goal", "collision", "truncated", "step", "episode")}
        assert torch.equal(ra, rb) and torch.equal(da, db)
    a.close()
    b.close()
