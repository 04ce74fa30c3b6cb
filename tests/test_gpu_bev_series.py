"""The 12-channel BEV option on the GPU (src/train.py:66 "(occupancy(MONO) + flow(RGB)) * series(3
steps)", :474-486 make_temporal_maps, src/gym_ffmp/envs/ffmp.py:16): ffmp_bev_image against the
oracle's bev_image bit for bit (the stated RGB encoding: parity unpinned against the reference, whose
encoding lived outside its repository); FFMPVec(bev_series=3).bev_maps() against the oracle env's
images fed through the reference's map_memory (TemporalStack, is_first = a reset); the replay
memory's BEV series against what the env emitted; Brain(input_channels=12) updating."""
import ctypes as C

import numpy as np
import pytest
import torch

from flow_field_based_motion_planner_amd import FFMPConfig, _abi
from flow_field_based_motion_planner_amd.replay import ReplayMemory
from flow_field_based_motion_planner_amd.vec_env import FFMPVec
from oracle.ffmp_oracle import Cfg, OracleVecEnv, Record, TemporalStack, bev_image, raster

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
CFG = FFMPConfig(grid=64, n_obst=8, n_beams=32, moving=True, max_steps=4, obst_rmax=0.5, obst_vmax=1.2,
                 world_half=3.2, goal_max=2.0, flow=True, seed=31)


def _direct(occ, flow, vmax, compact):
    n, plane = occ.shape[0], occ.shape[1]
    out = torch.full((n, 4, plane), 7, dtype=occ.dtype, device=DEV)
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    _abi.check(_abi.load().ffmp_bev_image(n, int(compact), occ.data_ptr(), plane, flow.data_ptr(), plane, vmax,
                                          out.data_ptr(), 4 * plane, s), "ffmp_bev_image")
    return out


@pytest.mark.parametrize("plane", [4096, 9801])  # 4 cells per thread / 1 (a plane not a multiple of 4)
@pytest.mark.parametrize("compact", [False, True])
def test_bev_image_equals_oracle(plane, compact):
    vmax = 1.2
    v = np.float32(vmax)
    rng = np.random.default_rng(plane + compact)
    n = 5
    fx = rng.uniform(-1.3, 1.3, (n, plane)).astype(np.float32) * v
    fy = rng.uniform(-1.3, 1.3, (n, plane)).astype(np.float32) * v
    # exact halves of the R / G / B grids, zero, +-vmax and beyond: the rounding mode's cases
    specials = np.array([0.0, v, -v, 2 * v, v / 255, v * 3 / 255, -v / 255, v / 510, -v / 510], np.float32)
    fx[:, :specials.size], fy[:, :specials.size] = specials, specials[::-1]
    occ = (rng.random((n, plane)) < 0.3).astype(np.float32) * 255
    flow = np.stack([fx, fy], 1)
    if compact:
        flow = flow.astype(np.float16)
        got = _direct(torch.as_tensor(occ.astype(np.uint8), device=DEV), torch.as_tensor(flow, device=DEV),
                      vmax, True).cpu().numpy().astype(np.float32)
    else:
        got = _direct(torch.as_tensor(occ, device=DEV), torch.as_tensor(flow, device=DEV), vmax, False).cpu().numpy()
    want = bev_image(occ.reshape(n, 1, plane), flow.astype(np.float32).reshape(n, 2, 1, plane), vmax)
    assert np.array_equal(got, want.reshape(n, 4, plane))


def _ref_images(ref, vmax, compact):
    flow = ref.flow.astype(np.float16).astype(np.float32) if compact else ref.flow
    return bev_image(ref.state_m[:, 1], flow, vmax)


@pytest.mark.parametrize("fmt,window", [("f32", 4), ("u8f16", 2)])
def test_bev_maps_match_reference_map_memory(fmt, window):
    n, steps, k = 24, 18, 3
    env = FFMPVec(n, CFG, device=DEV, frame_window=window, obs_format=fmt, autotune=False, bev_series=k)
    ref = OracleVecEnv(CFG, n)
    env.reset()
    ref.reset()
    stacks = {kk: [TemporalStack(kk) for _ in range(n)] for kk in (1, 2, 3)}

    def push(first):
        img = _ref_images(ref, CFG.obst_vmax, fmt == "u8f16")
        for kk, per_env in stacks.items():
            for e, st in enumerate(per_env):
                st.push(img[e], bool(first[e]))

    def check(tag):
        for kk, per_env in stacks.items():
            got = env.bev_maps(kk).cpu().numpy().astype(np.float32)
            want = np.stack([np.concatenate(st.mem, axis=0) for st in per_env])
            assert got.shape == (n, 4 * kk, 64, 64) and got.shape == want.shape
            bad = np.argwhere((got != want).any(axis=(2, 3)))
            assert bad.size == 0, f"{tag} k={kk}: (env, channel) mismatches {bad[:8].tolist()}"

    push(np.ones(n, bool))
    check("reset")
    rng = np.random.default_rng(4)
    resets = 0
    for s in range(steps):
        a = rng.integers(0, 28, n)
        env.step(torch.as_tensor(a, device=DEV))
        ref.step(a)
        push(ref.done)
        resets += int(ref.done.sum())
        check(f"step {s}")
    assert resets > n
    # a moving disc colours its cells: the flow channels are not constant
    img = env.bev_maps(1)
    assert int((img[:, 3] > 0).sum()) > 0 and int((img[:, 1] != 128).sum()) > 0
    with pytest.raises(ValueError):
        env.bev_maps(4)


def test_bev_maps_errors_and_reload():
    with pytest.raises(ValueError, match="flow=True"):
        FFMPVec(4, CFG.replace(flow=False), device=DEV, bev_series=3)
    env = FFMPVec(8, CFG, device=DEV, autotune=False, bev_series=3)
    with pytest.raises(RuntimeError, match="reset"):
        env.bev_maps(3)
    env.reset()
    for _ in range(2):
        env.step(torch.zeros(8, dtype=torch.int64, device=DEV))
    sd = env.state_dict()
    env2 = FFMPVec(8, CFG, device=DEV, autotune=False, bev_series=3)
    env2.load_state_dict(sd)
    assert torch.equal(env2.bev_maps(1), env.bev_maps(1))
    with pytest.raises(RuntimeError, match="known images"):
        env2.bev_maps(2)  # the older images are not part of a state_dict
    env2.step(torch.zeros(8, dtype=torch.int64, device=DEV))
    env.step(torch.zeros(8, dtype=torch.int64, device=DEV))
    assert torch.equal(env2.bev_maps(2), env.bev_maps(2))
    out = torch.empty(8, 8, 64, 64, device=DEV)
    assert env.bev_maps(2, out=out) is out
    with pytest.raises(ValueError):
        env.bev_maps(2, out=torch.empty(8, 4, 64, 64, device=DEV))


@pytest.mark.parametrize("obs_format", ["f32", "u8f16"])
def test_replay_bev_series_reproduces_the_env(obs_format):
    """ReplayMemory(series=3, bev=True): the state series re-rastered and coloured from the stored
    records equals env.bev_maps(3) before the step; the observation series equals it after the step,
    or for an env that reset, the state series slid by one with the terminal image appended.  In the
    compact layout the env colours binary16 flow planes, and so must the replay."""
    cfg = FFMPConfig(grid=64, n_obst=12, n_beams=32, moving=True, max_steps=5, obst_rmax=0.5, obst_vmax=1.2,
                     world_half=2.4, goal_min=0.6, goal_max=1.5, flow=True, seed=23)
    N, T, k = 32, 11, 3
    env = FFMPVec(N, cfg, device=DEV, keep_terminal=True, bev_series=k, obs_format=obs_format)
    mem = ReplayMemory(env, capacity=N * T, series=k, bev=True)
    env.reset()
    rng = np.random.default_rng(2)
    before, after, term, dones = [], [], [], []
    for _ in range(T):
        before.append(env.bev_maps(k).float())
        mem.push_begin()
        a = torch.as_tensor(rng.integers(0, 28, N), device=DEV)
        env.step(a)
        mem.push_end(a)
        after.append(env.bev_maps(k).float())
        term.append(env.term_record.clone())
        dones.append(env.done.clone())
    done_all = torch.cat(dones)
    assert 0 < int(done_all.sum()) < N * T
    tr, ex = mem.sample(0, index=torch.arange(N * T, device=DEV), potential=True)
    assert tr.state_m.shape == (N * T, 4 * k, 64, 64) and "flow" not in ex
    s_want = torch.cat(before)
    assert torch.equal(tr.state_m, s_want)
    nd = ~done_all
    assert torch.equal(tr.observe_m[nd], torch.cat(after)[nd])
    assert torch.equal(tr.observe_m[done_all][:, :-4], s_want[done_all][:, 4:])
    oc = Cfg.from_config(cfg)
    sm, _, flow = raster(oc, Record.unpack(torch.cat(term)[done_all].cpu().numpy(), cfg.n_obst), False)
    if obs_format == "u8f16":
        flow = flow.astype(np.float16).astype(np.float32)
    newest = bev_image(sm[:, 1], flow, cfg.obst_vmax)
    assert np.array_equal(tr.observe_m[done_all][:, -4:].cpu().numpy(), newest)
    mem2 = ReplayMemory(env, capacity=N * T, series=k, bev=True)
    mem2.load_state_dict(mem.state_dict())
    tr2, _ = mem2.sample(0, index=torch.arange(N * T, device=DEV))
    assert torch.equal(tr2.state_m, tr.state_m) and torch.equal(tr2.observe_m, tr.observe_m)
    with pytest.raises(ValueError):
        ReplayMemory(env, capacity=N * T, series=k).load_state_dict(mem.state_dict())


@pytest.mark.parametrize("amp", [False, True])
def test_brain_twelve_channels_updates(amp):
    from flow_field_based_motion_planner_amd.learner import Brain
    cfg = FFMPConfig(grid=100, n_obst=6, n_beams=0, moving=True, max_steps=20, flow=True, seed=41)
    n = 16
    env = FFMPVec(n, cfg, device=DEV, keep_terminal=True, bev_series=3, autotune=False)
    brain = Brain(env, capacity=256, batch_size=32, input_channels=12, amp=amp, seed=3)
    assert brain.main_q_network.conv1.in_channels == 12 and brain.memory.bev
    obs = env.reset()
    losses = []
    for _ in range(4):
        a = brain.decide_action(obs, env.episode)
        assert a.shape == (n,)
        brain.memory.push_begin()
        obs, _, _, _ = env.step(a)
        brain.memory.push_end(a)
        loss = brain.replay()
        if loss is not None:
            losses.append(float(loss))
    assert losses and all(np.isfinite(losses))
    with pytest.raises(ValueError, match="bev_series"):
        Brain(FFMPVec(n, cfg, device=DEV, keep_terminal=True, autotune=False), input_channels=12)


def test_bev_ring_counts_against_the_hbm_budget():
    """the BEV image ring is an arena buffer — a budget that holds the planes but not the
    ring is refused at construction, and an instance built within a budget holds the ring inside it."""
    cfg = FFMPConfig(grid=64, n_obst=4, n_beams=0, moving=True, max_steps=20, flow=True, seed=3)
    N, k = 4096, 3
    ring = k * N * 4 * 64 * 64 * 4  # 768 MiB
    planes = N * 64 * 64 * 4 * (2 + 1 + 2)  # frames (W = 2), potential, flow: 320 MiB
    with pytest.raises(ValueError):
        FFMPVec(N, cfg, device=DEV, bev_series=k, hbm_budget=planes + ring // 2, autotune=False)
    env = FFMPVec(N, cfg, device=DEV, bev_series=k, hbm_budget=planes + ring + (64 << 20), autotune=False)
    assert env.hbm_bytes() <= planes + ring + (64 << 20)
    a0 = env._arena_buf.data_ptr()
    assert a0 <= env.bev.data_ptr() < a0 + env._arena_buf.numel()
    env.reset()
    env.step(torch.zeros(N, dtype=torch.int64, device=DEV))
    assert env.bev_maps(k).shape == (N, 4 * k, 64, 64)
    env.close()
