"""Helpers shared by the GPU parity tests and tests/parity_report.py."""
from __future__ import annotations

import numpy as np

# Tolerances (north star: integer grid/obstacle indices bit-exact, float robot state <= 1e-5 abs).
EXACT_FIELDS = ("state_m", "done", "is_goal", "collision", "truncated", "t", "episode")
F64_STATE_ATOL = 1e-9      # pose / goal / obstacles / d0 (float64 state; 1e-5 is the contract)
F32_OBS_ATOL = 1e-5        # state_g, state_v, state_t, grad, reward, lidar (float32 obs)
POT_RTOL, POT_ATOL = 1e-6, 1e-5


def gpu_snapshot(env, sl=slice(None)):
    d = {k: getattr(env, k)[sl].detach().cpu().numpy() for k in
         ("state_m", "state_g", "state_v", "state_t", "grad", "reward", "done", "is_goal", "collision",
          "truncated", "pose", "goal", "d0", "obst", "obst_r", "t", "episode", "record")}
    d["potential"] = env.potential[sl].detach().cpu().numpy() if env.potential is not None else None
    d["lidar"] = env.lidar[sl].detach().cpu().numpy() if env.lidar is not None else None
    d["flow"] = env.flow[sl].detach().cpu().numpy() if env.flow is not None else None
    for k in ("term_record", "term_obs"):
        t = getattr(env, k, None)
        d[k] = t[sl].detach().cpu().numpy() if t is not None else None
    K = env.cfg.n_obst
    if K == 0:
        d["obst"] = d["obst"][:, :0]
        d["obst_r"] = d["obst_r"][:, :0]
    return d


def oracle_snapshot(ref):
    d = {k: getattr(ref, k) for k in
         ("state_m", "state_g", "state_v", "state_t", "grad", "reward", "done", "is_goal", "collision",
          "truncated", "pose", "goal", "d0", "obst", "obst_r", "t", "episode", "record")}
    d["potential"] = ref.potential if ref.with_potential else None
    d["lidar"] = ref.lidar if ref.cfg.n_beams else None
    d["flow"] = ref.flow
    d["term_record"] = getattr(ref, "term_record", None)
    d["term_obs"] = getattr(ref, "term_obs", None)
    return d


def compare(g, o, where=""):
    """Return a list of human-readable mismatch descriptions (empty == parity)."""
    bad = []

    def diff_count(a, b):
        a = np.asarray(a)
        b = np.asarray(b)
        if a.shape != b.shape:
            return f"shape {a.shape} vs {b.shape}"
        ne = ~((a == b) | (np.isnan(a) & np.isnan(b)) if a.dtype.kind == "f" else (a == b))
        return int(ne.sum())

    if (g.get("flow") is None) != (o.get("flow") is None):
        bad.append(f"{where} flow: present on one side only")
    elif g.get("flow") is not None and not np.array_equal(g["flow"], o["flow"]):
        bad.append(f"{where} flow: {int((g['flow'] != o['flow']).sum())} elements differ")
    if g.get("term_record") is not None:  # only envs built with keep_terminal have them
        c = diff_count(g["term_record"], o["term_record"])
        if c:
            bad.append(f"{where} term_record: {c} elements differ")
        a, b = np.asarray(g["term_obs"], dtype=np.float64), np.asarray(o["term_obs"], dtype=np.float64)
        if a.shape != b.shape or not np.allclose(a, b, rtol=0, atol=F32_OBS_ATOL):
            bad.append(f"{where} term_obs: mismatch")
    for k in EXACT_FIELDS + ("record",):
        c = diff_count(g[k], o[k])
        if c:
            bad.append(f"{where} {k}: {c} elements differ")
    for k in ("pose", "goal", "d0", "obst", "obst_r"):
        a, b = np.asarray(g[k], dtype=np.float64), np.asarray(o[k], dtype=np.float64)
        if a.shape != b.shape or not np.allclose(a, b, rtol=0, atol=F64_STATE_ATOL):
            bad.append(f"{where} {k}: max |diff| {np.max(np.abs(a - b)) if a.shape == b.shape else 'shape'}")
    for k in ("state_g", "state_v", "state_t", "grad", "reward", "lidar"):
        if g[k] is None and o[k] is None:
            continue
        a, b = np.asarray(g[k], dtype=np.float64), np.asarray(o[k], dtype=np.float64)
        same_inf = (np.isinf(a) & np.isinf(b) & (np.sign(a) == np.sign(b)))
        fa = np.where(same_inf, 0.0, a)
        fb = np.where(same_inf, 0.0, b)
        if a.shape != b.shape or not np.allclose(fa, fb, rtol=0, atol=F32_OBS_ATOL):
            m = np.max(np.abs(fa - fb)) if a.shape == b.shape else "shape"
            bad.append(f"{where} {k}: max |diff| {m}")
    if g["potential"] is not None:
        a, b = g["potential"], o["potential"]
        if not np.allclose(a, b, rtol=POT_RTOL, atol=POT_ATOL):
            bad.append(f"{where} potential: max |diff| {np.max(np.abs(a - b))}")
    return bad


def exact_report(g, o):
    """Count of non-bit-identical elements per float field (informational)."""
    out = {}
    for k in ("state_g", "state_v", "state_t", "grad", "reward", "lidar", "potential", "pose", "goal", "d0",
              "obst", "record"):
        if g.get(k) is None:
            continue
        a, b = np.asarray(g[k]), np.asarray(o[k])
        same = (a == b) | (np.isnan(a) & np.isnan(b))
        out[k] = int((~same).sum())
    return out


def env_like_stream(sc):
    """Split an env-like golden scenario into env steps: [(row, state_row_after_update)], skipping
    the reset-observation iterations (row 0 and each row after a done), which a batched env
    folds into the step that resets; returns (initial_state_row, steps)."""
    rows = sc["rows"]
    steps, k = [], 1
    while k < len(rows):
        r = rows[k]
        if r["done_out"]:
            if k + 1 >= len(rows):
                break
            steps.append((r, rows[k + 1]))
            k += 2
        else:
            steps.append((r, r))
            k += 1
    return rows[0], steps


def network_weights(shapes, seed=1234):
    """Deterministic float32 weights for the reference Network (name -> array), in state_dict
    order: weights ~ N(0, 1/fan_in), biases ~ N(0, 0.05^2).  numpy-only so the golden script and
    the GPU test build the same values on any machine."""
    rng = np.random.default_rng(seed)
    out = {}
    for name, shape in shapes:
        if name.endswith("weight"):
            fan_in = int(np.prod(shape[1:]))
            out[name] = (rng.standard_normal(shape) / np.sqrt(fan_in)).astype(np.float32)
        else:
            out[name] = (rng.standard_normal(shape) * 0.05).astype(np.float32)
    return out


def network_inputs(batch, seed):
    """Synthetic Network inputs at the reference map size (G=100): two 0/255 occupancy frames of
    random discs, relative goal, velocity and dt."""
    rng = np.random.default_rng(seed)
    G = 100
    yy, xx = np.mgrid[0:G, 0:G]
    sm = np.zeros((batch, 2, G, G), dtype=np.float32)
    for b in range(batch):
        for f in range(2):
            for _ in range(int(rng.integers(3, 9))):
                cx, cy, r = rng.uniform(0, G), rng.uniform(0, G), rng.uniform(2, 9)
                sm[b, f][(xx - cx) ** 2 + (yy - cy) ** 2 <= r * r] = 255.0
    g = np.stack([rng.uniform(0.5, 5.0, batch), rng.uniform(-np.pi, np.pi, batch)], 1).astype(np.float32)
    v = np.stack([rng.uniform(0, 0.06, batch), rng.uniform(-0.06, 0.06, batch)], 1).astype(np.float32)
    t = rng.uniform(0.0, 0.2, (batch, 1)).astype(np.float32)
    return sm, g, v, t

