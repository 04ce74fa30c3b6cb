"""Episode bookkeeping on the GPU (ffmp_episode_update through EpisodeTracker) against
  - the reference main loop's own statements (golden episode_bookkeeping, train.py:579-682),
    raw iteration streams and env-like streams (reset_iteration mode),
  - the oracle EpisodeBook on random flag streams (every field and the running totals, exact),
  - an FFMPVec stepping with auto-reset (tracker counters == env t / episode)."""
import numpy as np
import pytest
import torch

from flow_field_based_motion_planner_amd import EpisodeTracker, FFMPVec
from flow_field_based_motion_planner_amd.config import FFMPConfig
from oracle import ffmp_oracle as O
from tests.parity_util import env_like_stream

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _check_equal(tr, book):
    assert np.array_equal(tr.reach_rate.cpu().numpy(), book.reach_rate)
    assert np.array_equal(tr.step.cpu().numpy(), book.step)
    assert np.array_equal(tr.episode.cpu().numpy(), book.episode)
    assert np.array_equal(tr.total_step.cpu().numpy(), book.total_step)
    assert np.array_equal(tr.is_first.cpu().numpy(), book.is_first)
    assert np.array_equal(tr.complete.cpu().numpy(), book.complete)
    assert tr.totals.cpu().tolist() == book.totals.tolist()


@pytest.mark.parametrize("k", range(5))
def test_golden_scenarios_replicated(golden, k):
    """Each reference scenario replicated over 130 envs (two full waves and a ragged one)."""
    ep = golden["episode_bookkeeping"]
    sc = ep["scenarios"][k]
    n = 130
    tr = EpisodeTracker(n, window=ep["window"], threshold=ep["threshold"], max_steps=sc["max_steps"],
                        armed=sc["armed"], reset_iteration=False, device=DEV)
    for t, row in enumerate(sc["rows"]):
        assert bool(tr.is_first[0]) == row["first_in"]
        g = torch.full((n,), row["is_goal"], dtype=torch.bool, device=DEV)
        d = torch.full((n,), row["is_done_in"], dtype=torch.bool, device=DEV)
        tr.update(d, g, d & ~g)
        rr = tr.reach_rate.cpu().numpy()
        assert (rr == row["reach_rate"]).all(), (sc["name"], t)
        for name in ("episode", "step", "total_step"):
            assert (getattr(tr, name).cpu().numpy() == row[name]).all(), (sc["name"], t, name)
        assert (tr.complete.cpu().numpy() == row["is_complete"]).all()
        assert (tr.is_first.cpu().numpy() == row["is_first"]).all()
    s = tr.summary()
    assert s["env_steps"] == n * len(sc["rows"])
    assert s["episodes"] == n * sc["rows"][-1]["episode"]
    assert s["counted_steps"] == n * sc["rows"][-1]["total_step"]


def _rows_equal(tr, row, ctx):
    for name in ("reach_rate", "episode", "step", "total_step"):
        assert (getattr(tr, name).cpu().numpy() == row[name]).all(), (ctx, name)
    assert (tr.complete.cpu().numpy() == row["is_complete"]).all(), ctx
    assert (tr.is_first.cpu().numpy() == row["is_first"]).all(), ctx


@pytest.mark.parametrize("name", ["env_like", "env_like_goals"])
def test_golden_env_like_reset_iteration(golden, name):
    """Env steps only (the reset-observation iterations folded away) + reset_iteration=True
    reproduces the reference loop's counters row for row (70 envs, ragged wave)."""
    ep = golden["episode_bookkeeping"]
    sc = next(s for s in ep["scenarios"] if s["name"] == name)
    n = 70
    tr = EpisodeTracker(n, window=ep["window"], threshold=ep["threshold"], max_steps=sc["max_steps"], device=DEV)
    first, steps = env_like_stream(sc)
    _rows_equal(tr, first, "init")
    for t, (r, want) in enumerate(steps):
        d = torch.full((n,), r["is_done_in"], dtype=torch.bool, device=DEV)
        g = torch.full((n,), r["is_goal"], dtype=torch.bool, device=DEV)
        tr.update(d, g)
        _rows_equal(tr, want, (name, t))
    assert tr.summary()["episodes"] == n * sum(r["done_out"] for r, _ in steps)


@pytest.mark.parametrize("window,max_steps,armed,reset_it", [(10, 7, True, False), (64, 0, True, False),
                                                             (3, 4, False, True), (1, 2, True, False),
                                                             (10, 6, True, True)])
def test_random_streams_vs_oracle(window, max_steps, armed, reset_it):
    n, T = 1000, 40
    rng = np.random.default_rng(window * 100 + max_steps)
    thr = 0.3 if reset_it else 0.6  # with reset iterations the window holds at most one goal in two
    tr = EpisodeTracker(n, window=window, threshold=thr, max_steps=max_steps, armed=armed, reset_iteration=reset_it,
                        device=DEV)
    book = O.EpisodeBook(n, window=window, threshold=thr, max_steps=max_steps, armed=armed, reset_iteration=reset_it)
    _check_equal(tr, book)
    p_goal = rng.uniform(0.0, 0.9, n)  # per-env goal rates so some envs complete
    for t in range(T):
        u = rng.uniform(size=n)
        goal = u < p_goal
        col = (~goal) & (rng.uniform(size=n) < 0.1)
        trunc = (~goal) & (~col) & (rng.uniform(size=n) < 0.05)
        done = goal | col | trunc
        book.update(goal, done, col, trunc)
        tr.update(torch.from_numpy(done).to(DEV), torch.from_numpy(goal).to(DEV), torch.from_numpy(col).to(DEV),
                  torch.from_numpy(trunc).to(DEV))
        _check_equal(tr, book)
    assert book.totals[5] > 0 or not armed


def test_mask_init_and_checkpoint():
    n = 300
    tr = EpisodeTracker(n, window=10, max_steps=3, reset_iteration=False, device=DEV)
    ones = torch.ones(n, dtype=torch.bool, device=DEV)
    for _ in range(5):
        tr.update(~ones, ~ones)
    sd = tr.state_dict()
    mask = torch.zeros(n, dtype=torch.bool, device=DEV)
    mask[::3] = True
    tr.init(mask)
    st = tr.step.cpu().numpy()
    assert (st[::3] == 0).all() and (st[1::3] == sd["step"].cpu().numpy()[1::3]).all()
    assert tr.is_first.cpu().numpy()[::3].all() and not tr.is_first.cpu().numpy()[1::3].any()
    assert tr.totals.cpu().tolist() == sd["totals"].cpu().tolist()  # masked init keeps totals
    tr.load_state_dict(sd)
    assert torch.equal(tr.step, sd["step"])
    r = EpisodeTracker(n, device=DEV)  # reset_iteration: the first iteration is already done
    assert (r.step.cpu() == 1).all() and (r.total_step.cpu() == 1).all() and not r.is_first.any()
    assert (r.reach_len.cpu() == 1).all() and r.summary()["counted_steps"] == n
    with pytest.raises(ValueError):
        EpisodeTracker(4, window=65, device=DEV)
    with pytest.raises(ValueError):
        tr.update(ones[:10], ones[:10])


def test_tracks_vec_env():
    """Driving the tracker from FFMPVec flags: its step / episode counters follow the env's t /
    episode exactly (the env truncates at t == max_steps; tracker max_steps 0 or the same value)."""
    cfg = FFMPConfig(grid=64, n_obst=6, n_beams=64, moving=True, max_steps=9, goal_min=0.55, goal_max=0.65, seed=5)
    env = FFMPVec(777, cfg, device=DEV)
    env.reset()
    a = EpisodeTracker(777, max_steps=0, device=DEV)
    b = EpisodeTracker(777, max_steps=9, device=DEV)
    c = EpisodeTracker(777, max_steps=9, reset_iteration=False, device=DEV)
    g = torch.Generator(device="cpu").manual_seed(3)
    host = np.zeros(4, dtype=np.int64)  # done, goal, collision, truncated
    for _ in range(40):
        act = torch.randint(0, 28, (777,), generator=g).to(DEV)
        env.step(act)
        a.update_from(env)
        b.update_from(env)
        c.update_from(env)
        assert torch.equal(a.step, env.t + 1) and torch.equal(a.episode, env.episode)
        assert torch.equal(c.step, env.t) and torch.equal(c.episode, env.episode)
        host += [int(x.sum()) for x in (env.done, env.is_goal, env.collision, env.truncated)]
    for k, v in a.state_dict().items():
        assert torch.equal(v, getattr(b, k)), k
    s = a.summary()
    assert s["env_steps"] == 40 * 777 and s["episodes"] == int(env.episode.sum())
    assert [s["episodes"], s["goals"], s["collisions"], s["truncations"]] == host.tolist()
    assert s["counted_steps"] == int(a.total_step.sum()) == 41 * 777
    assert c.summary()["counted_steps"] == 40 * 777 - s["episodes"]
    assert min(host) > 0
