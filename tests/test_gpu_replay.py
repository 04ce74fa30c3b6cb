"""Device replay memory (replay.py): what sample() materialises is bit-identical to what the env
emitted (state before the step, observation after it — the terminal one for envs that reset),
and the ring follows the reference ReplayMemory's push / len / sample semantics
(src/train.py:212-228)."""
import numpy as np
import pytest
import torch

from flow_field_based_motion_planner_amd import FFMPConfig
from flow_field_based_motion_planner_amd.replay import ReplayMemory, Transition
from flow_field_based_motion_planner_amd.vec_env import FFMPVec
from oracle.ffmp_oracle import Cfg, Record, raster

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


class _RefRing:
    """src/train.py:212-228 ReplayMemory.push / __len__, restated over transition ids."""

    def __init__(self, capacity):
        self.capacity, self.memory, self.index = capacity, [], 0

    def push(self, item):
        if len(self.memory) < self.capacity:
            self.memory.append(None)
        self.memory[self.index] = item
        self.index = (self.index + 1) % self.capacity


def _snap(env):
    return {"state_m": env.state_m.clone(), "small": torch.cat([env.state_g, env.state_v, env.state_t], 1).clone(),
            "potential": env.potential.clone() if env.potential is not None else None,
            "flow": env.flow.clone() if env.flow is not None else None, "record": env.record.clone()}


@pytest.mark.parametrize("flow", [False, True])
def test_sample_reproduces_env_observations(flow):
    cfg = FFMPConfig(grid=64, n_obst=12, n_beams=32, moving=True, max_steps=5, obst_rmax=0.5, obst_vmax=1.2,
                     world_half=2.4, goal_min=0.6, goal_max=1.5, flow=flow, seed=21)
    N, T = 48, 9
    env = FFMPVec(N, cfg, device=DEV, keep_terminal=True)
    mem = ReplayMemory(env, capacity=N * T)
    env.reset()
    rng = np.random.default_rng(0)
    before, after, term, dones = [], [], [], []
    for _ in range(T):
        before.append(_snap(env))
        mem.push_begin()
        a = torch.as_tensor(rng.integers(0, 28, N), device=DEV)
        env.step(a)
        mem.push_end(a)
        after.append(_snap(env))
        term.append((env.term_record.clone(), env.term_obs.clone()))
        dones.append(env.done.clone())
    assert len(mem) == N * T
    done_all = torch.cat(dones)
    assert 0 < int(done_all.sum()) < N * T  # both kinds of transition are present
    idx = torch.arange(N * T, device=DEV)
    tr, ex = mem.sample(0, index=idx, potential=True)
    assert isinstance(tr, Transition) and tr.state_m.shape == (N * T, 2, 64, 64)
    assert tr.action.shape == (N * T, 1) and tr.reward.shape == (N * T,)
    assert torch.equal(tr.state_m, torch.cat([b["state_m"] for b in before]))
    assert torch.equal(ex["potential"], torch.cat([b["potential"] for b in before]))
    s_small = torch.cat([tr.state_g, tr.state_v, tr.state_t], 1)
    assert torch.equal(s_small, torch.cat([b["small"] for b in before]))
    o_small = torch.cat([tr.observe_g, tr.observe_v, tr.observe_t], 1)
    assert torch.equal(o_small, torch.cat([t[1] for t in term]))
    if flow:
        assert torch.equal(ex["flow"], torch.cat([b["flow"] for b in before]))
    # not-done transitions: observation == what the env returned after the step
    nd = ~done_all
    assert torch.equal(tr.observe_m[nd], torch.cat([a_["state_m"] for a_ in after])[nd])
    assert torch.equal(ex["observe_potential"][nd], torch.cat([a_["potential"] for a_ in after])[nd])
    assert torch.equal(o_small[nd], torch.cat([a_["small"] for a_ in after])[nd])
    assert torch.equal(ex["done"], done_all)
    # done transitions: the terminal frame (the oracle raster of the terminal record), not the reset one
    oc = Cfg.from_config(cfg)
    recs = torch.cat([t[0] for t in term])[done_all].cpu().numpy()
    sm_ref = raster(oc, Record.unpack(recs, cfg.n_obst), False)[0]
    got = tr.observe_m[done_all].cpu().numpy()
    assert np.array_equal(got, sm_ref)
    reset_frames = torch.cat([a_["state_m"] for a_ in after])[done_all].cpu().numpy()
    assert not np.array_equal(got, reset_frames)


def test_ring_semantics_and_sampling():
    cfg = FFMPConfig(grid=32, n_obst=4, n_beams=0, moving=True, max_steps=4, seed=22)
    N, cap, T = 16, 100, 10
    env = FFMPVec(N, cfg, device=DEV, keep_terminal=True)
    mem = ReplayMemory(env, capacity=cap, seed=5)
    ref = _RefRing(cap)
    env.reset()
    rng = np.random.default_rng(1)
    recs, acts = {}, {}
    for s in range(T):
        rec_before = env.record.clone()
        mem.push_begin()
        a = rng.integers(0, 28, N)
        env.step(torch.as_tensor(a, device=DEV))
        mem.push_end(torch.as_tensor(a, device=DEV))
        for e in range(N):
            ref.push((s, e))
            recs[(s, e)], acts[(s, e)] = rec_before[e], int(a[e])
        assert len(mem) == len(ref.memory) and mem.index == ref.index
    for slot, key in enumerate(ref.memory):
        assert torch.equal(mem.s_record[slot], recs[key]), slot
        assert int(mem.action[slot]) == acts[key]
    idx = mem.sample_indices(64)
    assert idx.unique().numel() == 64 and int(idx.max()) < cap
    assert mem.sample_indices(500, replacement=True).numel() == 500
    with pytest.raises(ValueError):
        mem.sample_indices(cap + 1)
    tr, ex = mem.sample(32)
    assert tr.state_m.shape == (32, 2, 32, 32) and ex["index"].unique().numel() == 32
    sd = mem.state_dict()
    mem2 = ReplayMemory(env, capacity=cap)
    mem2.load_state_dict(sd)
    tr2, _ = mem2.sample(32, index=ex["index"])
    assert torch.equal(tr2.state_m, tr.state_m) and torch.equal(tr2.observe_m, tr.observe_m)
    with pytest.raises(ValueError):
        ReplayMemory(FFMPVec(N, cfg, device=DEV), capacity=cap)  # needs keep_terminal
    with pytest.raises(RuntimeError):
        mem.push_end(torch.zeros(N, dtype=torch.int64, device=DEV))


@pytest.mark.parametrize("k", [3, 4])
def test_series_sample_reproduces_temporal_maps(k):
    """ReplayMemory(series=k): the k-frame state series re-rastered from the stored records equals
    env.temporal_maps(k) before the step; the observation series equals it after the step, or for
    an env that reset, the state series slid by one with the terminal frame appended (the reference
    appends the observed frame to map_memory; is_first refills it only on the next iteration)."""
    cfg = FFMPConfig(grid=64, n_obst=12, n_beams=32, moving=True, max_steps=5, obst_rmax=0.5, obst_vmax=1.2,
                     world_half=2.4, goal_min=0.6, goal_max=1.5, seed=23)
    N, T = 32, 11
    env = FFMPVec(N, cfg, device=DEV, keep_terminal=True, frame_window=k + 1)
    mem = ReplayMemory(env, capacity=N * T, series=k)
    env.reset()
    rng = np.random.default_rng(2)
    before, after, term, dones = [], [], [], []
    for _ in range(T):
        before.append(env.temporal_maps(k).clone())
        mem.push_begin()
        a = torch.as_tensor(rng.integers(0, 28, N), device=DEV)
        env.step(a)
        mem.push_end(a)
        after.append(env.temporal_maps(k).clone())
        term.append(env.term_record.clone())
        dones.append(env.done.clone())
    done_all = torch.cat(dones)
    assert 0 < int(done_all.sum()) < N * T
    tr, ex = mem.sample(0, index=torch.arange(N * T, device=DEV), potential=True)
    assert tr.state_m.shape == (N * T, k, 64, 64)
    s_want = torch.cat(before)
    assert torch.equal(tr.state_m, s_want)
    nd = ~done_all
    assert torch.equal(tr.observe_m[nd], torch.cat(after)[nd])
    assert torch.equal(tr.observe_m[done_all][:, :-1], s_want[done_all][:, 1:])
    oc = Cfg.from_config(cfg)
    recs = torch.cat(term)[done_all].cpu().numpy()
    newest = raster(oc, Record.unpack(recs, cfg.n_obst), False)[0][:, 1]
    assert np.array_equal(tr.observe_m[done_all][:, -1].cpu().numpy(), newest)
    sd = mem.state_dict()
    mem2 = ReplayMemory(env, capacity=N * T, series=k)
    mem2.load_state_dict(sd)
    tr2, _ = mem2.sample(0, index=torch.arange(N * T, device=DEV))
    assert torch.equal(tr2.state_m, tr.state_m) and torch.equal(tr2.observe_m, tr.observe_m)
