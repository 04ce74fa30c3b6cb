"""HIP path (through the C ABI) vs the NumPy oracle, step for step.

Tolerances (tests/parity_util.py): state_m, done/goal/collision/truncated, t,
episode and the raster record bit-exact; float64 state 1e-9 abs; float32 obs
1e-5 abs; potential rtol 1e-6 / atol 1e-5.
"""
import numpy as np
import pytest
import torch

from flow_field_based_motion_planner_amd import FFMPConfig, preset
from flow_field_based_motion_planner_amd.vec_env import FFMPVec
from oracle.ffmp_oracle import OracleVecEnv, Record, raster
from tests.parity_util import compare, exact_report, gpu_snapshot, oracle_snapshot

pytestmark = pytest.mark.gpu

CASES = {
    # name: (config, n_envs, steps)
    "C1_64_static": (FFMPConfig(grid=64, n_obst=4, n_beams=0, moving=False, max_steps=25, seed=1), 32, 30),
    "C2_128_static": (FFMPConfig(grid=128, n_obst=8, n_beams=0, moving=False, seed=2), 16, 12),
    "C3_256_moving_lidar": (FFMPConfig(grid=256, n_obst=16, n_beams=180, moving=True, max_steps=15, seed=3), 6, 18),
    "G100_reference_map": (FFMPConfig(grid=100, n_obst=4, n_beams=180, moving=False, seed=4), 16, 20),
    "dense_collisions": (FFMPConfig(grid=64, n_obst=64, n_beams=64, moving=True, obst_rmax=0.6, obst_vmax=1.5,
                                    world_half=3.2, goal_max=2.0, seed=5), 48, 40),
    "C5_512_moving_lidar": (FFMPConfig(grid=512, n_obst=32, n_beams=360, moving=True, seed=6), 2, 4),
    "no_obstacles": (FFMPConfig(grid=32, n_obst=0, n_beams=8, moving=False, max_steps=5, seed=7), 8, 12),
    "flow_planes": (FFMPConfig(grid=128, n_obst=24, n_beams=64, moving=True, flow=True, obst_rmax=0.7,
                               obst_vmax=1.2, seed=8), 12, 15),
}


def _run(cfg, n, steps, seed=0, env_offset=0, keep_terminal=True, frame_window=None, fused=None, fused_flags=None):
    env = FFMPVec(n, cfg, device="cuda:0", env_offset=env_offset, keep_terminal=keep_terminal,
                  frame_window=frame_window, fused=fused)
    if fused_flags is not None:
        env.fused_flags = fused_flags
    ref = OracleVecEnv(cfg, n, env_offset=env_offset)
    env.reset()
    ref.reset()
    torch.cuda.synchronize()
    problems = compare(gpu_snapshot(env), oracle_snapshot(ref), "reset")
    rng = np.random.default_rng(seed)
    counts = {"done": 0, "collision": 0, "goal": 0, "trunc": 0}
    for s in range(steps):
        a = rng.integers(0, 28, n)
        env.step(torch.as_tensor(a, device="cuda:0"))
        ref.step(a)
        torch.cuda.synchronize()
        g = gpu_snapshot(env)
        problems += compare(g, oracle_snapshot(ref), f"step {s}")
        counts["done"] += int(g["done"].sum())
        counts["collision"] += int(g["collision"].sum())
        counts["goal"] += int(g["is_goal"].sum())
        counts["trunc"] += int(g["truncated"].sum())
    return env, ref, problems, counts


@pytest.mark.parametrize("name", list(CASES))
def test_step_parity(name):
    cfg, n, steps = CASES[name]
    # half the cases keep the temporal stack in a 4-frame window (pair slides, wraps every 3 steps)
    window = 4 if name in ("C1_64_static", "dense_collisions", "flow_planes", "C3_256_moving_lidar") else 2
    env, ref, problems, counts = _run(cfg, n, steps, keep_terminal=name != "C2_128_static", frame_window=window)
    assert env.frame_window == window
    assert not problems, "\n".join(problems[:20])
    if name == "dense_collisions":
        assert counts["collision"] > 0 and counts["done"] > 0, counts  # the reset path is exercised


@pytest.mark.parametrize("name", ["C1_64_static", "C3_256_moving_lidar", "dense_collisions", "flow_planes",
                                  "G100_reference_map", "no_obstacles"])
def test_fused_step_parity(name):
    """The one-launch step (ffmp_step_fused: env step by wave 0, then the block's raster) against
    the oracle, through the seamless ring, with the 2-D tiles where the grid allows them."""
    from flow_field_based_motion_planner_amd import _abi
    cfg, n, steps = CASES[name]
    flags = _abi.RASTER_NT | _abi.RASTER_TILE4 | (_abi.RASTER_XCD if n >= 16 else 0)
    env, ref, problems, counts = _run(cfg, n, steps, frame_window=4, fused=True, fused_flags=flags)
    assert env.fused
    assert not problems, "\n".join(problems[:20])
    if name == "dense_collisions":
        assert counts["collision"] > 0 and counts["done"] > 0, counts


def test_fused_equals_two_launch_every_flag():
    """Every fused flag set writes the same planes and outputs as the two-launch step."""
    cfg = FFMPConfig(grid=128, n_obst=24, n_beams=40, moving=True, obst_rmax=0.7, obst_vmax=1.5, flow=True,
                     world_half=5.0, max_steps=5, seed=12)
    n = 21
    ref_env = FFMPVec(n, cfg, device="cuda:0", frame_window=3, fused=False)
    ref_env.reset()
    gen = torch.Generator(device="cuda:0").manual_seed(4)
    acts = torch.randint(0, 28, (8, n), device="cuda:0", generator=gen)
    want = []
    for k in range(8):
        o, r, d, _ = ref_env.step(acts[k], copy=True)
        want.append((o, r, d))
    for flags in FFMPVec.FUSED_FLAGS:
        env = FFMPVec(n, cfg, device="cuda:0", frame_window=3, fused=True)
        env.fused_flags = flags
        env.reset()
        for k in range(8):
            o, r, d, _ = env.step(acts[k])
            wo, wr, wd = want[k]
            assert torch.equal(d, wd) and torch.equal(r, wr), (flags, k)
            for key in ("state_m", "potential", "flow", "lidar", "state_g", "state_v", "grad"):
                assert torch.equal(o[key], wo[key]), (flags, k, key)


def test_truncation_and_autoreset_counts():
    cfg = FFMPConfig(grid=64, n_obst=0, n_beams=0, max_steps=3, goal_min=1.2, goal_max=1.2, seed=9)
    env, ref, problems, counts = _run(cfg, 4, 7)
    assert not problems
    assert counts["trunc"] == 2 * 4  # steps 3 and 6
    assert (env.episode.cpu().numpy() == 2).all()


def test_raster_parity_from_gpu_record():
    """Raster kernel alone: oracle raster of the GPU-written record == GPU planes, bit for bit."""
    cfg = FFMPConfig(grid=256, n_obst=32, n_beams=0, moving=True, obst_rmax=1.0, seed=11)
    env = FFMPVec(24, cfg, device="cuda:0")
    env.reset()
    rng = np.random.default_rng(1)
    for _ in range(3):
        env.step(torch.as_tensor(rng.integers(0, 28, 24), device="cuda:0"))
    torch.cuda.synchronize()
    rec = Record.unpack(env.record.cpu().numpy(), cfg.n_obst)
    from oracle.ffmp_oracle import Cfg
    sm, pot = raster(Cfg.from_config(cfg), rec)
    assert np.array_equal(env.state_m.cpu().numpy(), sm)
    assert np.array_equal(env.potential.cpu().numpy(), pot)


@pytest.mark.parametrize("G", [8, 12, 100, 124])
def test_raster_odd_sizes(G):
    """Grids whose G^2 is not a multiple of the 1024-cell pass (ragged tails)."""
    cfg = FFMPConfig(grid=G, n_obst=3, n_beams=4, moving=True, seed=G)
    env, ref, problems, _ = _run(cfg, 5, 4)
    assert not problems, "\n".join(problems[:10])


def test_shard_invariance_gpu():
    """Same global env index -> same trajectory whatever the shard layout."""
    cfg = FFMPConfig(grid=64, n_obst=8, n_beams=16, moving=True, seed=21)
    full = FFMPVec(12, cfg, device="cuda:0")
    a = FFMPVec(5, cfg, device="cuda:0", env_offset=0)
    b = FFMPVec(7, cfg, device="cuda:0", env_offset=5)
    for e in (full, a, b):
        e.reset()
    rng = np.random.default_rng(3)
    for _ in range(6):
        act = torch.as_tensor(rng.integers(0, 28, 12), device="cuda:0")
        full.step(act)
        a.step(act[:5])
        b.step(act[5:])
    torch.cuda.synchronize()
    for k in ("state_m", "pose", "reward", "lidar", "potential", "episode"):
        cat = torch.cat([getattr(a, k), getattr(b, k)])
        assert torch.equal(getattr(full, k), cat), k


def test_full_size_c3_properties():
    """BASELINE config C3 (32768 envs, 256^2, 16 moving discs, 180 beams): size-independent checks
    plus an oracle spot-check of individual env indices."""
    cfg = preset("C3", autoreset=True, seed=123)
    N = 32768
    env = FFMPVec(N, cfg, device="cuda:0")
    env.reset()
    gen = torch.Generator(device="cuda:0").manual_seed(0)
    acts = [torch.randint(0, 28, (N,), device="cuda:0", generator=gen) for _ in range(4)]
    prev_new = None
    for s, act in enumerate(acts):
        env.step(act)
        sm = env.state_m
        # values are exactly {0, 255}
        assert bool(((sm == 0) | (sm == 255)).all())
        # temporal stack: older frame == previous newest frame for envs that did not reset
        if prev_new is not None:
            keep = ~env.done
            assert torch.equal(sm[keep, 0], prev_new[keep])
            # reset envs start with a duplicated frame
            assert torch.equal(sm[env.done, 0], sm[env.done, 1])
        prev_new = sm[:, 1].clone()
        # gradient lookup == central difference of the potential plane at the robot cell
        G = cfg.grid
        c = G // 2
        P = env.potential
        inv = torch.tensor(np.float32(1.0 / (2.0 * cfg.res)), device="cuda:0")
        gx = (P[:, c + 1, c] - P[:, c - 1, c]) * inv
        gy = (P[:, c, c + 1] - P[:, c, c - 1]) * inv
        assert torch.equal(env.grad[:, 0], gx) and torch.equal(env.grad[:, 1], gy)
    torch.cuda.synchronize()
    # oracle spot-check of a few global env indices (shard invariance makes this exact)
    for idx in (0, 4097, N - 1):
        ref = OracleVecEnv(cfg, 1, env_offset=idx)
        ref.reset()
        for act in acts:
            ref.step(act[idx:idx + 1].cpu().numpy())
        g = gpu_snapshot(env, slice(idx, idx + 1))
        probs = compare(g, oracle_snapshot(ref), f"env {idx}")
        assert not probs, probs


def test_footprint_collision_consistent_with_frame():
    """With autoreset off, the footprint collision flag equals any(state_m[:,1][footprint] > 0)."""
    cfg = FFMPConfig(grid=64, n_obst=48, n_beams=0, moving=True, autoreset=False, obst_rmax=0.6,
                     world_half=3.2, goal_max=2.5, seed=31)
    env = FFMPVec(256, cfg, device="cuda:0")
    env.reset()
    rng = np.random.default_rng(4)
    c = cfg.grid // 2
    fp = cfg.footprint
    seen = 0
    for _ in range(10):
        env.step(torch.as_tensor(rng.integers(0, 28, 256), device="cuda:0"))
        fr = env.state_m[:, 1].cpu().numpy()
        foot = np.zeros(256, dtype=bool)
        for di, dj in fp:
            foot |= fr[:, c + di, c + dj] > 0
        assert np.array_equal(foot, env.collision.cpu().numpy())
        seen += int(foot.sum())
        env.reset(mask=env.done)
    assert seen > 0


def test_exactness_report(capsys):
    """Informational: how many float outputs are not bit-identical to the oracle."""
    cfg, n, steps = CASES["C3_256_moving_lidar"]
    env, ref, problems, _ = _run(cfg, n, 4)
    rep = exact_report(gpu_snapshot(env), oracle_snapshot(ref))
    print("non-bit-identical elements:", rep)
    assert rep["record"] == 0


@pytest.mark.parametrize("slices,window", [(2, None), (5, None), (3, 4), (2, 8)])
def test_pipelined_step_equals_serial(slices, window):
    """The two-stream pipelined step (env kernel of slice s+1 beside the raster of slice s)
    produces exactly the serial step's tensors — contiguous frames or the seamless ring (newest-only
    rasters per slice, the pair sliding through every slot incl. the alias)."""
    cfg = FFMPConfig(grid=64, n_obst=12, n_beams=32, moving=True, obst_rmax=0.5, seed=41)
    ser = FFMPVec(83, cfg, device="cuda:0", pipeline=1, frame_window=window)
    pip = FFMPVec(83, cfg, device="cuda:0", pipeline=slices, frame_window=window)
    assert pip.ring == ser.ring and (window is None or pip.ring == "seamless")
    assert pip.pipeline_slices == slices and ser.pipeline_slices == 1
    ser.reset()
    pip.reset()
    gen = torch.Generator(device="cuda:0").manual_seed(5)
    for _ in range(19):
        a = torch.randint(0, 28, (83,), device="cuda:0", generator=gen)
        t1, t2 = [], []
        ser.step(a, timing=t1)
        pip.step(a, timing=t2)
        assert len(t1) == 1 and len(t2) == slices and sum(r[2] for r in t2) == 83
        assert torch.equal(ser.state_m, pip.state_m)
    torch.cuda.synchronize()
    g1, g2 = gpu_snapshot(ser), gpu_snapshot(pip)
    for k in g1:
        if g1[k] is not None:
            assert np.array_equal(g1[k], g2[k]), k


def test_raster_shapes_identical():
    """Every launch shape the autotuner may pick writes bit-identical planes."""
    from flow_field_based_motion_planner_amd import _abi
    cfg = FFMPConfig(grid=128, n_obst=24, n_beams=0, moving=True, obst_rmax=0.8, seed=77)
    env = FFMPVec(37, cfg, device="cuda:0", autotune=False)
    env.reset()
    env.step(torch.randint(0, 28, (37,), device="cuda:0"))
    ref = None
    extra = ((1024, 0), (3072, _abi.RASTER_XCD), (8192, 0), (1024, _abi.RASTER_TILE4),
             (3072, _abi.RASTER_TILE8 | _abi.RASTER_XCD), (2048, _abi.RASTER_TILE2), (1024, _abi.RASTER_TILE8))
    for shape in FFMPVec.RASTER_SHAPES + extra:
        env.state_m.fill_(-1.0)
        env.potential.fill_(-1.0)
        env.raster_shape = shape
        env.raster()
        got = (env.state_m.clone(), env.potential.clone())
        if ref is None:
            ref = got
        assert torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1]), shape


@pytest.mark.parametrize("grid", [256, 96, 100, 512, 192])
def test_tile_shapes_identical_with_flow(grid):
    """2-D wave tiles (R = 2, 4, 8) write the same frames, potential and flow planes as the
    256-cell chunks, in full and newest-only launches (G = 96: only R = 8 tiles apply; G = 100:
    none does, the chunks run)."""
    from flow_field_based_motion_planner_amd import _abi
    cfg = FFMPConfig(grid=grid, n_obst=32, n_beams=0, moving=True, obst_rmax=0.6, obst_vmax=1.5, flow=True,
                     world_half=grid * 0.05 * 0.75, max_steps=4, seed=grid)
    shapes = [(2048, 0), (2048, _abi.RASTER_TILE2), (2048, _abi.RASTER_TILE4), (4096, _abi.RASTER_TILE8),
              (16384, _abi.RASTER_TILE4 | _abi.RASTER_NT), (8192, _abi.RASTER_TILE4 | _abi.RASTER_XCD)]
    ref = None
    for shape in shapes:
        env = FFMPVec(11, cfg, device="cuda:0", autotune=False, frame_window=4)
        env.raster_shape = env.raster_shape_newest = shape
        env.reset()
        gen = torch.Generator(device="cuda:0").manual_seed(3)
        outs = []
        for _ in range(7):
            o, _, _, _ = env.step(torch.randint(0, 28, (11,), device="cuda:0", generator=gen))
            outs.append((o["state_m"].clone(), o["potential"].clone(), o["flow"].clone()))
        if ref is None:
            ref = outs
        for got, want in zip(outs, ref):
            for a, b in zip(got, want):
                assert torch.equal(a, b), shape


def test_newest_only_shapes_identical():
    """Newest-only launches (frame ring) are bit-identical for every shape, too."""
    cfg = FFMPConfig(grid=64, n_obst=24, n_beams=0, moving=True, obst_rmax=0.8, max_steps=3, seed=78)
    ref = None
    for shape in FFMPVec.RASTER_SHAPES:
        env = FFMPVec(29, cfg, device="cuda:0", autotune=False, frame_window=5)
        env.raster_shape = env.raster_shape_newest = shape
        env.reset()
        gen = torch.Generator(device="cuda:0").manual_seed(9)
        outs = []
        for _ in range(9):
            o, _, _, _ = env.step(torch.randint(0, 28, (29,), device="cuda:0", generator=gen))
            outs.append((o["state_m"].clone(), o["potential"].clone()))
        if ref is None:
            ref = outs
        for (a, b), (c, d) in zip(outs, ref):
            assert torch.equal(a, c) and torch.equal(b, d), shape


def test_autotune_picks_a_candidate():
    cfg = FFMPConfig(grid=128, n_obst=8, n_beams=0, seed=3)
    env = FFMPVec(8192, cfg, device="cuda:0")  # 8192 x 3 x 64 KiB planes > AUTOTUNE_MIN_BYTES
    assert env.placement is not None
    assert tuple(env.raster_shape) in FFMPVec.RASTER_SHAPES
    assert env.frame_window == 8 and tuple(env.raster_shape_newest) in FFMPVec.RASTER_SHAPES
    with pytest.raises(RuntimeError):
        env.step(torch.zeros(8192, dtype=torch.int64, device="cuda:0"))  # autotune leaves it un-reset
    env.reset()
    env.step(torch.zeros(8192, dtype=torch.int64, device="cuda:0"))


@pytest.mark.parametrize("ring", ["seamless", "seamless-slot0", "wrap"])
@pytest.mark.parametrize("window", [3, 4, 8])
def test_frame_window_equals_contiguous(window, ring):
    """The in-place temporal stack (frame window W: newest-only rasters, plus wraps for the
    wrapping ring; the seamless ring's virtual slot W is slot 0 again) yields the same
    observations, bit for bit, as rewriting both frames every step (W = 2), across resets."""
    cfg = FFMPConfig(grid=64, n_obst=24, n_beams=16, moving=True, obst_rmax=0.6, obst_vmax=1.5, world_half=3.0,
                     max_steps=7, flow=True, seed=41)
    n = 40
    a = FFMPVec(n, cfg, device="cuda:0", frame_window=2)
    slot0 = ring == "seamless-slot0"  # the wrap step writes slot 0 through its own addresses
    ring = "seamless" if slot0 else ring
    b = FFMPVec(n, cfg, device="cuda:0", frame_window=window, seamless=ring == "seamless")
    b.WRAP_VIA_ALIAS = not slot0
    assert b.ring == ring and a.ring == "contiguous"
    if ring == "seamless":  # slot W is a second mapping of slot 0 (padded slot stride)
        assert b.frames.shape[0] == window + 1 and b.frames.stride(0) >= n * 64 * 64
        assert b.frames[window].data_ptr() != b.frames[0].data_ptr()
    assert not b.state_m.is_contiguous() and b.state_m.shape == a.state_m.shape
    a.reset()
    b.reset()
    assert torch.equal(a.state_m, b.state_m)
    rng = np.random.default_rng(window)
    resets = 0
    for s in range(3 * window + 5):
        act = torch.as_tensor(rng.integers(0, 28, n), device="cuda:0")
        oa, _, da, _ = a.step(act)
        ob, _, db, _ = b.step(act)
        resets += int(da.sum())
        assert torch.equal(oa["state_m"], ob["state_m"]), s
        assert torch.equal(oa["potential"], ob["potential"]) and torch.equal(oa["flow"], ob["flow"])
        assert torch.equal(da, db)
        if s == window:  # masked reset mid-window
            m = torch.zeros(n, dtype=torch.bool, device="cuda:0")
            m[::5] = True
            a.reset(mask=m)
            b.reset(mask=m)
            assert torch.equal(a.state_m, b.state_m)
    assert resets > 0
    if ring == "seamless":
        assert torch.equal(b.frames[window], b.frames[0])
        b.frames[window, 3, 5, 7] = 17.0  # a write through the alias is seen through slot 0
        torch.cuda.synchronize()
        assert float(b.frames[0, 3, 5, 7]) == 17.0
    sd = b.state_dict()  # checkpoint round trip re-rasters the current pair in place
    b.state_m.fill_(-1.0)
    b.load_state_dict(sd)
    assert torch.equal(a.state_m, b.state_m)



def test_limits_parity():
    """The ABI's maxima at once: K = 64 discs, L = 1024 beams, a 1024^2 grid, global env indices
    above 2^32 (the Philox counter's high word), a 3-frame ring — against the oracle."""
    cfg = FFMPConfig(grid=1024, n_obst=64, n_beams=1024, moving=True, max_steps=4, obst_rmax=0.8,
                     obst_vmax=1.5, seed=2 ** 63 + 12345)
    env, ref, problems, counts = _run(cfg, 3, 6, env_offset=2 ** 32 + 7, frame_window=3)
    assert not problems, "\n".join(problems[:10])
    assert counts["done"] > 0


def test_single_env_and_ragged_counts():
    """n = 1 and n not a multiple of the 4-env / 64-lane groupings, through the ring."""
    for n in (1, 3, 65, 130):
        cfg = FFMPConfig(grid=32, n_obst=5, n_beams=70, moving=True, max_steps=3, seed=n)
        env, ref, problems, _ = _run(cfg, n, 5, frame_window=4)
        assert not problems, (n, problems[:5])


def test_no_potential_same_frames():
    """Without a potential plane the raster skips the potential math and culls with the
    occupancy reach only: frames (and flow) stay bit-identical to the full raster's."""
    cfg = FFMPConfig(grid=64, n_obst=24, n_beams=8, moving=True, obst_rmax=0.6, obst_vmax=1.5, world_half=3.0,
                     max_steps=6, flow=True, seed=43)
    for w in (2, 4):
        a = FFMPVec(33, cfg, device="cuda:0", frame_window=w)
        b = FFMPVec(33, cfg, device="cuda:0", frame_window=w, potential=False)
        a.reset()
        b.reset()
        rng = np.random.default_rng(w)
        for _ in range(10):
            act = torch.as_tensor(rng.integers(0, 28, 33), device="cuda:0")
            oa, _, _, _ = a.step(act)
            ob, _, _, _ = b.step(act)
            assert torch.equal(oa["state_m"], ob["state_m"]) and torch.equal(oa["flow"], ob["flow"])
            assert "potential" not in ob


@pytest.mark.parametrize("K,lanes_list", [(12, (16, 32, 64)), (16, (4, 8, 16, 32, 64)), (24, (16, 8, 32, 64))])
def test_env_lanes_identical(K, lanes_list):
    """Every lanes-per-env layout of env_kernel — 1, 2, 4 envs per wave with one disc per lane, and
    (round 4) 8 or 16 envs per wave with 2 or 4 discs per lane — gives the same state, observations
    and flags, bit for bit, through resets (and matches the oracle)."""
    from flow_field_based_motion_planner_amd import _abi
    cfg = FFMPConfig(grid=64, n_obst=K, n_beams=40, moving=True, obst_rmax=0.5, obst_vmax=1.2, world_half=2.6,
                     max_steps=5, seed=44)
    snaps = {}
    try:
        for lanes in lanes_list:
            _abi.set_tuning(_abi.TUNE_ENV_LANES, lanes)
            env, ref, problems, counts = _run(cfg, 23, 10, frame_window=3)
            assert not problems, (lanes, problems[:5])
            assert counts["done"] > 0
            snaps[lanes] = gpu_snapshot(env)
    finally:
        _abi.set_tuning(_abi.TUNE_ENV_LANES, 0)
    first = snaps[lanes_list[0]]
    for lanes in lanes_list[1:]:
        for k in first:
            if first[k] is not None:
                assert np.array_equal(first[k], snaps[lanes][k], equal_nan=True), (lanes, k)


def test_env_layout_falls_back_when_the_lds_does_not_fit():
    """4 waves per block x 16 envs per wave (4 lanes, 4 discs per lane) at L = 1024 would
    need 256 KiB of beam minima per block; the launch takes a layout that fits instead of failing,
    and the results equal the default layout's and the oracle's."""
    from flow_field_based_motion_planner_amd import _abi
    cfg = FFMPConfig(grid=32, n_obst=16, n_beams=1024, moving=True, obst_rmax=0.5, obst_vmax=1.2, world_half=1.6,
                     goal_max=1.2, max_steps=5, seed=45)
    snaps = {}
    for waves, lanes in ((1, 0), (4, 4)):
        pw, pl = _abi.set_tuning(_abi.TUNE_ENV_WAVES, waves), _abi.set_tuning(_abi.TUNE_ENV_LANES, lanes)
        try:
            env, ref, problems, counts = _run(cfg, 37, 6, frame_window=3)
        finally:
            _abi.set_tuning(_abi.TUNE_ENV_WAVES, pw)
            _abi.set_tuning(_abi.TUNE_ENV_LANES, pl)
        assert not problems, (waves, lanes, problems[:5])
        snaps[(waves, lanes)] = gpu_snapshot(env)
    a, b = snaps[(1, 0)], snaps[(4, 4)]
    for k in a:
        if a[k] is not None:
            assert np.array_equal(a[k], b[k], equal_nan=True), k
