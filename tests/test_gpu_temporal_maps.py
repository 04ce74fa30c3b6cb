"""make_temporal_maps over k frames (src/train.py:474-486 with INPUT_CHANNELS = k mono frames,
:66-69) served from the frame ring by ffmp_temporal_maps, against the oracle's TemporalStack fed
with the oracle env's newest frames (is_first = the step's auto-reset, or the initial reset).
Bit-exact: the frames are 0/255 bytes or floats copied, never computed."""
import numpy as np
import pytest
import torch

from flow_field_based_motion_planner_amd import FFMPConfig
from flow_field_based_motion_planner_amd.vec_env import FFMPVec
from oracle.ffmp_oracle import OracleVecEnv, TemporalStack

pytestmark = pytest.mark.gpu

# short episodes (max_steps 4) and dense discs: resets at every lag position of the window
CFG = FFMPConfig(grid=64, n_obst=8, n_beams=32, moving=True, max_steps=4, obst_rmax=0.5, obst_vmax=1.2,
                 world_half=3.2, goal_max=2.0, seed=11)


def _stacks(ref, ks):
    return {k: [TemporalStack(k) for _ in range(ref.n)] for k in ks}


def _push(stacks, ref, first):
    for k, per_env in stacks.items():
        for e, st in enumerate(per_env):
            st.push(ref.state_m[e, 1:2].copy(), bool(first[e]))


def _check(env, stacks, tag):
    for k, per_env in stacks.items():
        got = env.temporal_maps(k).cpu().numpy().astype(np.float32)
        want = np.stack([np.concatenate(st.mem, axis=0) for st in per_env])
        assert got.shape == want.shape, (tag, k, got.shape, want.shape)
        bad = np.argwhere((got != want).any(axis=(2, 3)))
        assert bad.size == 0, f"{tag} k={k}: (env, channel) mismatches {bad[:8].tolist()}"


@pytest.mark.parametrize("window,seamless,fmt", [(4, True, "f32"), (6, True, "u8f16"), (5, False, "f32"),
                                                 (2, False, "f32")])
def test_temporal_maps_match_reference_stack(window, seamless, fmt):
    n, steps = 24, 22
    env = FFMPVec(n, CFG, device="cuda:0", frame_window=window, seamless=seamless if window > 2 else None,
                  obs_format=fmt, autotune=False)
    assert env.ring == ("contiguous" if window == 2 else "seamless" if seamless else "wrap")
    ref = OracleVecEnv(CFG, n)
    env.reset()
    ref.reset()
    # a wrapping ring keeps W - 1 frames once it has wrapped: k = W is refused up front,
    # not after the first wrap
    ks = [k for k in range(1, window + 1) if window == 2 or seamless or k < window]
    assert env.max_temporal_frames == max(ks)
    if env.ring == "wrap":
        with pytest.raises(ValueError, match="wrapping ring"):
            env.temporal_maps(window)
    stacks = _stacks(ref, ks)
    _push(stacks, ref, np.ones(n, bool))
    _check(env, stacks, "reset")
    rng = np.random.default_rng(3)
    resets = 0
    for s in range(steps):
        a = rng.integers(0, 28, n)
        env.step(torch.as_tensor(a, device="cuda:0"))
        ref.step(a)
        assert np.array_equal(env.state_m.cpu().numpy().astype(np.float32), ref.state_m), f"state_m step {s}"
        _push(stacks, ref, ref.done)
        resets += int(ref.done.sum())
        _check(env, stacks, f"step {s}")
    assert resets > n, resets  # episodes end at every lag position


def test_temporal_maps_masked_reset_and_reload():
    n, W = 16, 5
    env = FFMPVec(n, CFG.replace(max_steps=0), device="cuda:0", frame_window=W, autotune=False)
    ref = OracleVecEnv(CFG.replace(max_steps=0), n)
    env.reset()
    ref.reset()
    stacks = _stacks(ref, [3, 5])
    _push(stacks, ref, np.ones(n, bool))
    rng = np.random.default_rng(5)
    for s in range(7):
        a = rng.integers(0, 28, n)
        env.step(torch.as_tensor(a, device="cuda:0"))
        ref.step(a)
        _push(stacks, ref, ref.done)
    mask = np.zeros(n, bool)
    mask[::3] = True
    env.reset(mask=torch.as_tensor(mask, device="cuda:0"))
    ref.reset(mask=mask)
    for per_env in stacks.values():  # a masked reset is a new first frame of those envs only
        for e in np.flatnonzero(mask):
            per_env[e].push(ref.state_m[e, 1:2].copy(), True)
    _check(env, stacks, "masked reset")
    # a reload re-rasters the [older, newest] pair only: deeper lags are refused until stepped again
    sd = env.state_dict()
    env2 = FFMPVec(n, CFG.replace(max_steps=0), device="cuda:0", frame_window=W, autotune=False)
    env2.load_state_dict(sd)
    assert torch.equal(env2.temporal_maps(2), env.temporal_maps(2))
    with pytest.raises(RuntimeError):
        env2.temporal_maps(3)
    for s in range(3):
        a = rng.integers(0, 28, n)
        env2.step(torch.as_tensor(a, device="cuda:0"))
        ref.step(a)
        _push(stacks, ref, ref.done)
    _check(env2, stacks, "after reload")


def test_temporal_maps_out_and_errors():
    n = 8
    env = FFMPVec(n, CFG, device="cuda:0", frame_window=4, autotune=False)
    env.reset()
    env.step(torch.zeros(n, dtype=torch.int64, device="cuda:0"))
    out = torch.empty(n, 4, 64, 64, device="cuda:0")
    assert env.temporal_maps(4, out=out).data_ptr() == out.data_ptr()
    # k = 2 through the kernel equals the state_m view
    o2 = torch.empty(n, 2, 64, 64, device="cuda:0")
    assert torch.equal(env.temporal_maps(2, out=o2), env.state_m)
    with pytest.raises(ValueError):
        env.temporal_maps(5)
    with pytest.raises(ValueError):
        env.temporal_maps(3, out=torch.empty(n, 3, 64, 64, device="cuda:0", dtype=torch.float16))
