"""Independent geometric checks of the rows the reference does not pin (SURVEY §8a a15-a19:
unicycle integrator, obstacle motion, occupancy raster, potential field, lidar).  The oracle and
the HIP path share one SPEC, so their bit-equality alone cannot catch a SPEC-level
mistake; these checks restate each output as a geometric property computed a different way, in
float64 from world coordinates, and apply it to the oracle (CPU) and to the HIP path (GPU):

  * lidar — a finite range R puts the hit point on a disc surface or a world wall, and the segment
    before it meets no disc (point-to-segment distances, no ray-quadratic); +inf: no disc and no
    wall within lidar_max; -inf: the sensor is inside a disc;
  * occupancy — cell (i, j) of the newest frame is 255 iff its world position (pose + R(yaw) · ego)
    is inside a disc or outside the world (cells within 1e-4 m of a boundary skipped: float32);
  * potential — 0.5 k_att |c - g|^2 + sum 0.5 k_rep (1/rho - 1/rho0)^2 over discs with
    rho = max(|c - o| - r, rho_min) < rho0, from world geometry (atol 2e-2 + rtol 1e-4: float32
    ego coordinates against a steep term near rho_min);
  * integrator — x' = x + v cos(yaw) dt, y' = y + v sin(yaw) dt, yaw' = wrap(yaw + w dt) with the
    reference's literal command table, for envs that did not reset (1e-12);
  * obstacle motion — each coordinate advances by v dt or is mirrored off its wall |p| = W - r with
    that velocity component negated; parked discs stay.
"""
import math

import numpy as np
import pytest

from flow_field_based_motion_planner_amd.config import FFMPConfig

V_CMD = (0.0, 0.2, 0.4, 0.6)                     # src/gym_ffmp/envs/robot/config.py:28-55
W_CMD = (-0.6, -0.4, -0.2, 0.0, 0.2, 0.4, 0.6)


def _wrap(a):
    a = np.array(a, dtype=np.float64)
    while np.any(a >= math.pi):
        a = np.where(a >= math.pi, a - 2 * math.pi, a)
    while np.any(a <= -math.pi):
        a = np.where(a <= -math.pi, a + 2 * math.pi, a)
    return a


def _seg_dist(px, py, ax, ay, bx, by):
    """Distance from points (px, py) to the segment a-b (broadcast)."""
    dx, dy = bx - ax, by - ay
    L2 = dx * dx + dy * dy
    t = np.clip(((px - ax) * dx + (py - ay) * dy) / np.where(L2 > 0, L2, 1.0), 0.0, 1.0)
    qx, qy = ax + t * dx - px, ay + t * dy - py
    return np.sqrt(qx * qx + qy * qy)


def check_lidar(cfg: FFMPConfig, pose, ox, oy, orr, lidar, tol=1e-4):
    bad = []
    n, L = lidar.shape
    W, Lmax = cfg.W, cfg.lidar_range
    live = orr > 0
    for e in range(n):
        x, y, yaw = pose[e]
        d2 = (ox[e] - x) ** 2 + (oy[e] - y) ** 2
        inside = bool(np.any(live[e] & (d2 <= orr[e] ** 2)))
        surface = bool(np.any(live[e] & (np.abs(np.sqrt(d2) - orr[e]) < tol)))
        for l in range(L):
            R = float(lidar[e, l])
            if inside:
                if R != -np.inf:
                    bad.append(f"env {e} beam {l}: sensor inside a disc but range {R}")
                continue
            if R == -np.inf:
                if not surface:
                    bad.append(f"env {e} beam {l}: -inf but the sensor is outside every disc")
                continue
            a = yaw + (-math.pi + l * 2 * math.pi / L)
            dx, dy = math.cos(a), math.sin(a)
            reach = Lmax if R == np.inf else R - tol
            ex, ey = x + reach * dx, y + reach * dy
            # the segment before the hit (or the whole range) meets no disc ...
            dseg = _seg_dist(ox[e], oy[e], x, y, ex, ey)
            if np.any(live[e] & (dseg < orr[e] - tol)):
                k = int(np.argmax(live[e] & (dseg < orr[e] - tol)))
                bad.append(f"env {e} beam {l}: range {R} passes through disc {k}")
                continue
            # ... and stays inside the world
            if abs(ex) > W + tol or abs(ey) > W + tol:
                bad.append(f"env {e} beam {l}: range {R} passes the world wall")
                continue
            if R == np.inf:
                continue
            if not (0 < R <= Lmax + tol):
                bad.append(f"env {e} beam {l}: range {R} outside (0, lidar_max]")
                continue
            hx, hy = x + R * dx, y + R * dy  # the hit point lies on a surface
            on_disc = np.any(live[e] & (np.abs(np.hypot(hx - ox[e], hy - oy[e]) - orr[e]) < 10 * tol))
            on_wall = abs(abs(hx) - W) < 10 * tol or abs(abs(hy) - W) < 10 * tol
            if not (on_disc or on_wall):
                bad.append(f"env {e} beam {l}: hit point ({hx:.5f}, {hy:.5f}) of range {R} is on no surface")
    return bad


def _cells_world(cfg, pose_e):
    G, res = cfg.grid, cfg.res
    half = 0.5 * G * res
    idx = np.arange(G, dtype=np.float64) * res - half
    ex, ey = np.meshgrid(idx, idx, indexing="ij")   # row i = ego x, column j = ego y
    x, y, yaw = pose_e
    c, s = math.cos(yaw), math.sin(yaw)
    return ex, ey, x + c * ex - s * ey, y + s * ex + c * ey


def check_occupancy(cfg, pose, ox, oy, orr, frame, tol=1e-4):
    bad = []
    W = cfg.W
    for e in range(frame.shape[0]):
        _, _, wx, wy = _cells_world(cfg, pose[e])
        occ = (np.abs(wx) > W) | (np.abs(wy) > W)
        near = (np.abs(np.abs(wx) - W) < tol) | (np.abs(np.abs(wy) - W) < tol)
        for k in range(ox.shape[1]):
            if orr[e, k] <= 0:
                continue
            d = np.hypot(wx - ox[e, k], wy - oy[e, k])
            occ |= d <= orr[e, k]
            near |= np.abs(d - orr[e, k]) < tol
        got = frame[e] != 0
        if not np.all(np.isin(frame[e], (0, 255))):
            bad.append(f"env {e}: cell values other than 0 / 255")
        wrong = (got != occ) & ~near
        if wrong.any():
            i, j = np.argwhere(wrong)[0]
            bad.append(f"env {e}: {int(wrong.sum())} cells disagree, first ({i}, {j}) got {frame[e, i, j]}")
    return bad


def check_potential(cfg, pose, goal, ox, oy, orr, pot):
    bad = []
    rho_min = cfg.res / 2 if cfg.rho_min is None else cfg.rho_min
    for e in range(pot.shape[0]):
        _, _, wx, wy = _cells_world(cfg, pose[e])
        U = 0.5 * cfg.k_att * ((wx - goal[e, 0]) ** 2 + (wy - goal[e, 1]) ** 2)
        for k in range(ox.shape[1]):
            rho = np.maximum(np.hypot(wx - ox[e, k], wy - oy[e, k]) - orr[e, k], rho_min)
            U = U + np.where(rho < cfg.rho0, 0.5 * cfg.k_rep * (1.0 / rho - 1.0 / cfg.rho0) ** 2, 0.0)
        err = np.abs(pot[e].astype(np.float64) - U)
        lim = 2e-2 + 1e-4 * np.abs(U)
        if np.any(err > lim):
            i, j = np.unravel_index(int(np.argmax(err - lim)), err.shape)
            bad.append(f"env {e}: potential off by {err[i, j]:.3g} at ({i}, {j}) ({pot[e, i, j]} vs {U[i, j]:.6g})")
    return bad


def check_integrator(cfg, pose0, pose1, actions, reset):
    a = np.asarray(actions)
    v = np.array([V_CMD[i // 7] for i in a])
    w = np.array([W_CMD[i % 7] for i in a])
    x0, y0, yaw0 = pose0[:, 0], pose0[:, 1], pose0[:, 2]
    want = np.stack([x0 + (v * np.cos(yaw0)) * cfg.dt, y0 + (v * np.sin(yaw0)) * cfg.dt, _wrap(yaw0 + w * cfg.dt)], 1)
    keep = ~np.asarray(reset)
    err = np.abs(pose1[keep] - want[keep])
    return [] if err.size == 0 or err.max() <= 1e-12 else [f"integrator off by {err.max():.3g}"]


def check_obstacle_motion(cfg, obst0, obst1, orr, reset, tol=1e-12):
    """Moving discs: each coordinate advances by v dt, or is mirrored off the wall |p| = W - r
    (the overshoot folded back inside, that velocity component negated); speed is preserved;
    parked discs (r = 0) and static configs stay put."""
    bad = []
    keep = ~np.asarray(reset)
    W, dt = cfg.W, cfg.dt
    for ax in (0, 1):
        p0, v0, p1, v1 = obst0[..., ax], obst0[..., 2 + ax], obst1[..., ax], obst1[..., 2 + ax]
        if not cfg.moving:
            ok = (p1 == p0) & (v1 == v0)
        else:
            free = p0 + v0 * dt
            lim = W - orr
            mirrored = np.where(free > lim, 2 * lim - free, np.where(free < -lim, -2 * lim - free, free))
            flipped = np.where((free > lim) | (free < -lim), -v0, v0)
            moving = orr > 0
            ok = np.where(moving, (np.abs(p1 - mirrored) <= tol) & (v1 == flipped) & (np.abs(p1) <= lim + tol),
                          (p1 == p0) & (v1 == v0))
        if not np.all(ok[keep]):
            e, k = np.argwhere(~ok & keep[:, None])[0]
            bad.append(f"env {e} disc {k} axis {ax}: {p0[e, k]} + {v0[e, k]} dt -> {p1[e, k]}, v {v1[e, k]}")
    return bad


CFG = FFMPConfig(grid=64, n_obst=12, n_beams=90, moving=True, obst_rmax=0.5, obst_vmax=1.0, world_half=2.4,
                 max_steps=8, seed=21)


def _check_all(cfg, pose0, actions, pose1, goal, obst, obst_r, lidar, state_m, pot, done, obst0=None):
    ox, oy = obst[..., 0], obst[..., 1]
    problems = check_integrator(cfg, pose0, pose1, actions, done)
    if obst0 is not None:
        problems += check_obstacle_motion(cfg, obst0, obst, obst_r, done)
    problems += check_lidar(cfg, pose1, ox, oy, obst_r, lidar)
    problems += check_occupancy(cfg, pose1, ox, oy, obst_r, state_m[:, 1])
    problems += check_potential(cfg, pose1, goal, ox, oy, obst_r, pot)
    return problems


def test_spec_geometry_oracle():
    from oracle.ffmp_oracle import OracleVecEnv
    n = 12
    env = OracleVecEnv(CFG, n)
    env.reset()
    rng = np.random.default_rng(5)
    hits = finite = resets = 0
    for _ in range(10):
        a = rng.integers(0, 28, n)
        pose0, obst0 = env.pose.copy(), env.obst.copy()
        env.step(a)
        problems = _check_all(CFG, pose0, a, env.pose, env.goal, env.obst, env.obst_r, env.lidar, env.state_m,
                              env.potential, env.done, obst0)
        assert not problems, "\n".join(problems[:10])
        hits += int((env.state_m[:, 1] != 0).sum())
        finite += int(np.isfinite(env.lidar).sum())
        resets += int(env.done.sum())
    assert hits > 0 and finite > 0 and resets > 0  # the checks saw walls, discs and resets


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,n", [(CFG, 24),
                                   (FFMPConfig(grid=256, n_obst=16, n_beams=180, moving=True, max_steps=6, seed=3), 8)])
def test_spec_geometry_hip(cfg, n):
    import torch
    from flow_field_based_motion_planner_amd.vec_env import FFMPVec
    env = FFMPVec(n, cfg, device="cuda:0")
    env.reset()
    gen = torch.Generator(device="cuda:0").manual_seed(6)
    acts = torch.randint(0, 28, (8, n), device="cuda:0", generator=gen)
    finite = 0
    for k in range(8):
        pose0, obst0 = env.pose.cpu().numpy(), env.obst.cpu().numpy()
        obs, _, done, _ = env.step(acts[k])
        torch.cuda.synchronize()
        problems = _check_all(cfg, pose0, acts[k].cpu().numpy(), env.pose.cpu().numpy(), env.goal.cpu().numpy(),
                              env.obst.cpu().numpy(), env.obst_r.cpu().numpy(), obs["lidar"].cpu().numpy(),
                              obs["state_m"].cpu().numpy(), obs["potential"].cpu().numpy(), done.cpu().numpy(), obst0)
        assert not problems, "\n".join(problems[:10])
        finite += int(torch.isfinite(obs["lidar"]).sum())
    assert finite > 0
