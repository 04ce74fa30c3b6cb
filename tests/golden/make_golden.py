#!/usr/bin/env python3
"""Generate the golden vectors that pin the oracle to the reference.

RUNS ONLY IN THE BUILD CONTAINER (it needs /root/reference, which never travels
to the GPU box).  It imports the reference's own code at run time and records
INPUTS and OUTPUTS only; no reference source is copied into this repository.

What is driven (reference file:line):
  * gym_ffmp.envs.ffmp.FFMP  (src/gym_ffmp/envs/ffmp.py:22-188)
      is_collision (:85-105; also at map widths that are not multiples of 4, differ from
      map_grid_num or are not square), is_collision2 (:108-117), is_goal (:120-127),
      reward_calculator (:130-157, incl. the module-global d0 and the
      NameError before the first is_first), is_done (:160-164),
      rewarder (:167-176), rewarder2 (:179-188)
  * RobotAction.cmd (src/gym_ffmp/envs/robot/config.py:25-58)
  * train.py helpers, compiled from the reference file's AST without importing
    rospy: ROSNode.pi_to_pi (:167-172), relative_goal_calculator (:174-180),
    robot_velocity_calculator (:182-188), Environment.make_temporal_maps
    (:474-486).
  * train.py Network (:231-303), compiled from the AST and run on CPU with deterministic
    numpy weights (tests/parity_util.network_weights) on synthetic G=100 inputs at B=1 and B=3
    (B>1 pins the batch coupling of the fc1 tile, :261-267).
  * train.py main-loop episode bookkeeping (:579-587 reach_times / reach_rate,
    :593 is_first, :606-607 truncation, :611-682 the is_done branch with its
    episode / step / total_step counters and the reach-rate completion test),
    compiled from the loop's own statements and driven with scripted
    (is_goal, is_done) sequences; ROS, TensorBoard, CSV and torch.save are
    inert stand-ins (unittest.mock), so only the bookkeeping runs.

`gym` is not installed here (nor on the GPU box), so a minimal offline stand-in
(this file's own code: Env, spaces.Box/Dict, envs.registration.register) is
written to a temp dir and put on sys.path before the reference is imported.

Usage:  python tests/golden/make_golden.py      (writes ref_pinned.json, ref_maps.npz)
"""
import ast
import contextlib
import copy
import io
import json
import math
import os
import sys
import tempfile
import types

import numpy as np

REF_SRC = "/root/reference/src"
OUT_DIR = os.path.dirname(os.path.abspath(__file__))

_GYM_STANDIN = {
    "gym/__init__.py": (
        "from . import spaces, error, utils, envs\n"
        "class Env(object):\n"
        "    pass\n"
        "def make(env_id):\n"
        "    return envs.registration._REG[env_id]()\n"
    ),
    "gym/error.py": "",
    "gym/utils/__init__.py": "from . import seeding\n",
    "gym/utils/seeding.py": "",
    "gym/envs/__init__.py": "from . import registration\n",
    "gym/envs/registration.py": (
        "_REG = {}\n"
        "def register(id, entry_point, **kw):\n"
        "    mod, name = entry_point.split(':')\n"
        "    def _mk():\n"
        "        import importlib\n"
        "        return getattr(importlib.import_module(mod), name)()\n"
        "    _REG[id] = _mk\n"
    ),
    "gym/spaces.py": (
        "import numpy as np\n"
        "class Box(object):\n"
        "    def __init__(self, low, high, dtype=np.float32, shape=None):\n"
        "        self.low = np.asarray(low); self.high = np.asarray(high); self.dtype = dtype\n"
        "        self.shape = self.low.shape\n"
        "class Dict(object):\n"
        "    def __init__(self, d):\n"
        "        self.spaces = dict(d)\n"
    ),
}


def _install_gym_standin():
    root = tempfile.mkdtemp(prefix="gym_standin_")
    for rel, txt in _GYM_STANDIN.items():
        p = os.path.join(root, rel)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "w") as f:
            f.write(txt)
    sys.path.insert(0, root)
    sys.path.insert(0, REF_SRC)


def _train_helpers():
    """Compile four helper methods out of the reference train.py AST."""
    import torch
    with open(os.path.join(REF_SRC, "train.py")) as f:
        tree = ast.parse(f.read())
    want = {("ROSNode", "pi_to_pi"), ("ROSNode", "relative_goal_calculator"),
            ("ROSNode", "robot_velocity_calculator"), ("Environment", "make_temporal_maps")}
    fns = []
    for node in tree.body:
        if isinstance(node, ast.ClassDef):
            for sub in node.body:
                if isinstance(sub, ast.FunctionDef) and (node.name, sub.name) in want:
                    fns.append(sub)
    mod = ast.Module(body=fns, type_ignores=[])
    g = {"math": math, "np": np, "copy": copy, "torch": torch, "INPUT_CHANNELS": 2}
    exec(compile(mod, "<reference train.py helpers>", "exec"), g)
    return g


def _episode_block():
    """The bookkeeping statements of train.py's main loop, compiled from its AST."""
    with open(os.path.join(REF_SRC, "train.py")) as f:
        src = f.read()
    tree = ast.parse(src)
    loop = next(n for n in ast.walk(tree) if isinstance(n, ast.While) and "is_shutdown" in ast.unparse(n.test))
    body = next(n for n in loop.body if isinstance(n, ast.If) and "is_start_callback_flag" in ast.unparse(n.test)).body

    def keep(st):
        txt = ast.unparse(st)
        head = txt.splitlines()[0]
        return (head in ("if is_goal:", "if len(reach_times) > REACH_MEMORY_CAPACITY:", "if step == MAX_STEPS:",
                         "if is_done:", "is_first = False")
                or head.startswith("train_env.reach_rate = "))

    stmts = [st for st in body if keep(st)]
    assert len(stmts) == 6, [ast.unparse(s_).splitlines()[0] for s_ in stmts]
    return compile(ast.Module(body=stmts, type_ignores=[]), "<reference train.py episode bookkeeping>", "exec"), \
        [st.lineno for st in stmts]


def _run_episode_block(events, max_steps, armed, n=None):
    """Drive the compiled bookkeeping with (is_goal, is_done) per loop iteration; `events` is a
    list, or a function of the previous iteration's row (None first) returning the next event."""
    from unittest import mock
    code, _ = _episode_block()
    train_env = mock.MagicMock()
    train_env.agent.brain.loss = mock.MagicMock() if armed else None
    g = {"np": np, "torch": mock.MagicMock(), "print": lambda *a, **k: None,
         "MAX_STEPS": max_steps, "REACH_MEMORY_CAPACITY": 10, "REACH_RATE_THRESHOLD": 0.80,
         "UPDATE_TARGET_EPISODE": 2, "MODEL_PATH": "/nonexistent/model.pth",
         "ros": mock.MagicMock(), "tensor_board": mock.MagicMock(), "writer": mock.MagicMock(),
         "train_env": train_env, "episode": 0, "step": 0, "total_step": 0, "reach_times": np.empty(0),
         "is_first": True, "is_complete": False, "numpy_reward": 0.0, "reward": 0.0,
         "relative_goal": np.zeros(2), "action_id": 3, "observe_m": None, "observe_g": None,
         "observe_v": None, "observe_t": None}
    rows = []
    seq = events if not callable(events) else (events(rows[-1] if rows else None) for _ in range(n))
    for goal, done in seq:
        first_in = g["is_first"]
        g["is_goal"], g["is_done"] = bool(goal), bool(done)
        exec(code, g)
        rows.append({"is_goal": bool(goal), "is_done_in": bool(done), "first_in": bool(first_in),
                     "reach_rate": float(train_env.reach_rate), "episode": int(g["episode"]),
                     "step": int(g["step"]), "total_step": int(g["total_step"]),
                     "is_complete": bool(g["is_complete"]), "is_first": bool(g["is_first"])})
    return rows


def _network_outputs(out, maps):
    import torch
    import torch.nn as nn
    import torch.nn.functional as F
    sys.path.insert(0, os.path.dirname(os.path.dirname(OUT_DIR)))
    from tests.parity_util import network_inputs, network_weights
    with open(os.path.join(REF_SRC, "train.py")) as f:
        tree = ast.parse(f.read())
    cls = next(n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == "Network")
    g = {"torch": torch, "nn": nn, "F": F, "BATCH_SIZE": 1024, "device": torch.device("cpu")}
    exec(compile(ast.Module(body=[cls], type_ignores=[]), "<reference train.py Network>", "exec"), g)
    torch.manual_seed(0)
    net = g["Network"](2, 28)
    sd = net.state_dict()
    w = network_weights([(k, tuple(v.shape)) for k, v in sd.items()])
    net.load_state_dict({k: torch.from_numpy(v) for k, v in w.items()})
    net.eval()
    res = {"weights": "tests/parity_util.network_weights(seed=1234)", "param_shapes": [[k, list(v.shape)] for k, v in
                                                                                       sd.items()], "cases": []}
    for batch, seed in ((1, 71), (3, 72), (2, 73)):
        sm, gg, vv, tt = network_inputs(batch, seed)
        with torch.no_grad(), contextlib.redirect_stdout(io.StringIO()):
            q = net(torch.from_numpy(sm), torch.from_numpy(gg), torch.from_numpy(vv), torch.from_numpy(tt))
        res["cases"].append({"batch": batch, "seed": seed, "q": q.numpy().astype(float).tolist()})
    out["network"] = res


class _Pose(object):
    def __init__(self, x, y, yaw):
        self.x, self.y, self.yaw = x, y, yaw


def main():
    _install_gym_standin()
    import gym_ffmp  # noqa: F401  (registers FFMP-v0 with the stand-in)
    from gym_ffmp.envs import ffmp as ffmp_mod
    from gym_ffmp.envs.ffmp import FFMP
    from gym_ffmp.envs.robot.config import RobotAction

    rng = np.random.default_rng(20240601)
    out = {"generator": "tests/golden/make_golden.py", "reference": "YoshitakaNagai/flow_field_based_motion_planner"}
    maps = {}

    # ---- NameError before the first is_first (must run before any reward call) ----
    env = FFMP()
    try:
        env.reward_calculator(np.array([1.0, 0.0]), False, False, False)
        out["reward_nameerror"] = False
    except NameError:
        out["reward_nameerror"] = True

    # ---- module constants / spaces ----
    out["constants"] = {
        "MAP_RANGE": ffmp_mod.MAP_RANGE, "MAP_GRID_NUM": ffmp_mod.MAP_GRID_NUM,
        "ROBOT_RSIZE": ffmp_mod.ROBOT_RSIZE, "MAP_RESOLUTION": ffmp_mod.MAP_RESOLUTION,
        "GOAL_THRESHOLHD": ffmp_mod.GOAL_THRESHOLHD,
        "action_low": env.action_low.tolist(), "action_high": env.action_high.tolist(),
        "goal_high": env.goal_high.tolist(),
    }
    act = RobotAction()
    out["action_table"] = [[c.linear_v, c.angular_v] for c in act.cmd]

    # ---- footprint cells for several G (generalised map_range = G * res) ----
    out["footprint"] = {}
    for G in (64, 100, 128, 256, 512):
        e = FFMP()
        if G != 100:
            e.map_grid_num = G
            e.map_range = G * ffmp_mod.MAP_RESOLUTION
        e.is_collision(np.zeros((G, G), dtype=np.int32))
        out["footprint"][str(G)] = [[int(c[0]), int(c[1])] for c in e.robot_grids]

    # ---- is_collision: single-cell window maps at G in {64,100,128} ----
    out["is_collision_single"] = {}
    for G in (64, 100, 128):
        e = FFMP()
        if G != 100:
            e.map_grid_num = G
            e.map_range = G * ffmp_mod.MAP_RESOLUTION
        c = G // 2
        res = []
        for i in range(c - 4, c + 5):
            for j in range(c - 4, c + 5):
                m = np.zeros((G, G), dtype=np.int32)
                m[i, j] = 255
                res.append([i, j, bool(e.is_collision(m))])
        out["is_collision_single"][str(G)] = res

    # ---- is_collision: random sparse maps at G=100 (2-D and (G,G,1) layouts) ----
    e = FFMP()
    rmaps, rres = [], []
    for k in range(48):
        dens = [0.0005, 0.002, 0.01, 0.05][k % 4]
        m = (rng.random((100, 100)) < dens).astype(np.int32) * rng.integers(1, 256, (100, 100))
        if k % 6 == 0:  # force a hit right on a footprint boundary cell
            m[50 + 2, 50 + 1] = 7
        rmaps.append(m.astype(np.uint8))
        r2d = bool(e.is_collision(m.astype(np.int32)))
        r3d = bool(e.is_collision(m.astype(np.int32)[:, :, None]))
        rres.append([r2d, r3d])
    maps["is_collision_maps"] = np.stack(rmaps)
    out["is_collision_random"] = rres

    # ---- is_collision2 on scan lists ----
    f13 = float(np.float32(0.13))
    f13_up = float(np.nextafter(np.float32(0.13), np.float32(1)))
    hand = [
        [None], [None, 0.5, 1.0], [None, 0.13], [None, f13], [None, f13_up],
        [None, 0.0, 0.0, 0.2], [None, 0.0, 0.12], [0.12999999999999998], [0.13000000000000003],
        [None, float("inf"), 0.3], [None, float("-inf")], [None, float("nan"), 0.2],
        [], [None, 0.05, 0.01],
    ]
    scans = []
    for s in hand:
        with contextlib.redirect_stdout(io.StringIO()) as buf:
            r = bool(e.is_collision2(s))
        scans.append({"scan": s, "collide": r, "printed": buf.getvalue()})
    for k in range(40):
        L = [180, 360][k % 2]
        v = rng.uniform(0.125, 6.0, L).astype(np.float32)
        if k % 3 == 0:
            v[rng.integers(0, L)] = np.float32(rng.choice([0.13, 0.1299, 0.1301, 0.12999999]))
        if k % 5 == 0:
            v[rng.integers(0, L, 4)] = 0.0
        s = [None] + [float(x) for x in v]
        with contextlib.redirect_stdout(io.StringIO()):
            r = bool(e.is_collision2(s))
        scans.append({"scan": s, "collide": r})
    out["is_collision2"] = scans

    # ---- is_goal ----
    gv = [0.0, 0.49999999999999994, 0.5, 0.5000000000000001, 1.0, -1.0, 0.25]
    gv += [float(x) for x in rng.uniform(0.3, 0.7, 40)]
    out["is_goal"] = [[d, bool(e.is_goal(d))] for d in gv]

    # ---- is_done ----
    out["is_done"] = [[a, b, bool(e.is_done(a, b))] for a in (False, True) for b in (False, True)]

    # ---- reward_calculator episode sequences (module-global d0) ----
    seqs = []
    for k in range(30):
        steps = []
        n = int(rng.integers(2, 12))
        d = float(rng.uniform(1.0, 6.0))
        for t in range(n):
            first = t == 0
            col = bool(rng.random() < 0.1)
            goal = bool(rng.random() < 0.1)
            orient = float(rng.uniform(-math.pi, math.pi))
            rg = np.array([d, orient])
            r = e.reward_calculator(rg, col, goal, first)
            steps.append({"rel_goal": [d, orient], "col": col, "goal": goal, "first": first,
                          "reward": float(r), "rtype": type(r).__name__})
            d = float(max(0.0, d + rng.uniform(-0.1, 0.08)))
        seqs.append(steps)
    out["reward_sequences"] = seqs
    # cross-instance leak of the module global
    a, b = FFMP(), FFMP()
    a.reward_calculator(np.array([3.0, 0.0]), False, False, True)
    leak = b.reward_calculator(np.array([2.5, 0.0]), False, False, False)
    out["reward_global_leak"] = {"d0_from_other_instance": 3.0, "d": 2.5, "reward": float(leak)}

    # ---- rewarder (map) and rewarder2 (scan) composites ----
    rw = []
    for k in range(24):
        m = maps["is_collision_maps"][k].astype(np.int32)
        rg = np.array([float(rng.uniform(0.2, 4.0)), float(rng.uniform(-3, 3))])
        first = (k % 4 == 0)
        r, done = e.rewarder(m, rg, first)
        rw.append({"map_index": k, "rel_goal": rg.tolist(), "first": first, "reward": float(r), "done": bool(done)})
    out["rewarder"] = rw
    rw2 = []
    for k in range(24):
        s = scans[(k * 3) % len(scans)]["scan"]
        rg = np.array([float(rng.uniform(0.2, 4.0)), float(rng.uniform(-3, 3))])
        first = (k % 4 == 0)
        with contextlib.redirect_stdout(io.StringIO()):
            r, done, goal = e.rewarder2(s, rg, first)
        rw2.append({"scan_index": (k * 3) % len(scans), "rel_goal": rg.tolist(), "first": first,
                    "reward": float(r), "done": bool(done), "is_goal": bool(goal)})
    out["rewarder2"] = rw2

    # ---- train.py helpers ----
    h = _train_helpers()
    ros = types.SimpleNamespace()
    ros.pi_to_pi = types.MethodType(h["pi_to_pi"], ros)
    angles = [0.0, math.pi, -math.pi, 3 * math.pi, -3 * math.pi, 2 * math.pi, -2 * math.pi, 7.0, -7.0,
              math.pi - 1e-15, -math.pi + 1e-15, 1e-300, -1e-300, 4.0, -4.0]
    angles += [float(x) for x in np.linspace(-20.0, 20.0, 161)]
    angles += [float(x) for x in rng.uniform(-12.0, 12.0, 100)]
    out["pi_to_pi"] = [[a, ros.pi_to_pi(a)] for a in angles]

    ros.global_goal = types.SimpleNamespace(position=types.SimpleNamespace(x=0.0, y=0.0))
    ros.relative_goal_calculator = types.MethodType(h["relative_goal_calculator"], ros)
    rel = []
    for k in range(120):
        gx, gy = (float(v) for v in rng.uniform(-12, 12, 2))
        px, py = (float(v) for v in rng.uniform(-12, 12, 2))
        yaw = float(rng.uniform(-math.pi, math.pi))
        if k < 4:
            gx, gy, px, py = [(1.0, 0.0, 0.0, 0.0), (0.0, 0.0, 0.0, 0.0), (-1.0, 0.0, 0.0, 0.0), (0.0, -2.0, 0.0, 0.0)][k]
        ros.global_goal.position.x, ros.global_goal.position.y = gx, gy
        r = ros.relative_goal_calculator(_Pose(px, py, yaw))
        rel.append({"goal": [gx, gy], "pose": [px, py, yaw], "out": [float(r[0]), float(r[1])]})
    out["relative_goal"] = rel

    ros.pre_robot_pose = _Pose(0.0, 0.0, 0.0)
    ros.robot_velocity_calculator = types.MethodType(h["robot_velocity_calculator"], ros)
    vel = []
    x, y, yaw = 0.0, 0.0, 0.0
    for k in range(80):
        first = (k % 10 == 0)
        if first:
            x, y, yaw = (float(v) for v in rng.uniform(-3, 3, 3))
        else:
            x += float(rng.uniform(-0.06, 0.06))
            y += float(rng.uniform(-0.06, 0.06))
            yaw = float(ros.pi_to_pi(yaw + float(rng.uniform(-0.6, 0.6))))
        r = ros.robot_velocity_calculator(_Pose(x, y, yaw), first)
        vel.append({"pose": [x, y, yaw], "first": first, "out": [float(r[0]), float(r[1])]})
    out["velocity"] = vel

    import torch
    tenv = types.SimpleNamespace(map_memory=[])
    tenv.make_temporal_maps = types.MethodType(h["make_temporal_maps"], tenv)
    tm = []
    for k in range(7):
        first = k in (0, 4)
        frame = torch.full((1, 3, 3), float(k))
        with contextlib.redirect_stdout(io.StringIO()):
            st = tenv.make_temporal_maps(frame, first)
        tm.append({"frame_value": float(k), "first": first, "stack": st[:, 0, 0].tolist(), "shape": list(st.shape)})
    out["temporal_maps"] = tm

    # ---- train.py Network ----
    _network_outputs(out, maps)

    # ---- train.py main-loop episode bookkeeping ----
    ep = {"block_lines": _episode_block()[1], "window": 10, "threshold": 0.80, "scenarios": []}
    for name, n, p_goal, p_col, max_steps, armed in (("mixed", 120, 0.15, 0.10, 6, True),
                                                     ("goal_rich", 80, 0.85, 0.05, 6, True),
                                                     ("goal_rich_unarmed", 60, 0.85, 0.05, 6, False),
                                                     ("truncation_only", 40, 0.0, 0.0, 4, True),
                                                     ("window_edge", 30, 0.5, 0.0, 200, True)):
        u = rng.uniform(size=n)
        events = [(bool(x < p_goal), bool(x < p_goal + p_col)) for x in u]
        ep["scenarios"].append({"name": name, "max_steps": max_steps, "armed": armed,
                                "rows": _run_episode_block(events, max_steps, armed)})
    # env-like streams: every episode starts with the iteration that observes the freshly reset
    # world (never at the goal, never colliding), as in a simulator driven by this loop
    for name, n, p_goal, p_col, max_steps in (("env_like", 150, 0.12, 0.08, 5), ("env_like_goals", 100, 0.6, 0.0, 9)):
        def env_event(prev, p_goal=p_goal, p_col=p_col):
            if prev is None or prev["is_first"]:  # the iteration that observes the reset world
                return (False, False)
            x = float(rng.uniform())
            return (x < p_goal, x < p_goal + p_col)

        rows = _run_episode_block(env_event, max_steps, True, n)
        prev = 0
        for r in rows:  # the iteration's final is_done (incl. the :607 truncation)
            r["done_out"], prev = r["episode"] != prev, r["episode"]
        ep["scenarios"].append({"name": name, "max_steps": max_steps, "armed": True, "env_like": True, "rows": rows})
    out["episode_bookkeeping"] = ep

    # ---- is_collision at the edges: map widths that are not multiples of 4 or
    # differ from map_grid_num, non-square maps, and instance attributes that move the footprint.
    # The reference indexes the ABSOLUTE cells of its footprint list (ffmp.py:87-101), in list order,
    # breaking at the first occupied one: a cell outside the given map raises IndexError only when it
    # is reached before a hit.  Own RNG: the draws above are unchanged.
    erng = np.random.default_rng(20261018)
    edge, emaps = [], {}
    cases = [  # (instance map_grid_num or None = default, map shape)
        (None, (50, 50)), (None, (98, 98)), (None, (99, 99)), (None, (100, 60)), (None, (60, 100)),
        (None, (53, 53)), (None, (101, 101)), (64, (100, 100)), (64, (37, 37)), (128, (100, 100)),
        (128, (66, 66)), (40, (50, 50)),
    ]
    for ci, (mg, shape) in enumerate(cases):
        e = FFMP()
        if mg is not None:
            e.map_grid_num = mg
            e.map_range = mg * ffmp_mod.MAP_RESOLUTION
        e.is_collision(np.zeros((120, 120), dtype=np.int32))  # the footprint cells of these attributes
        cells = [(int(c[0]), int(c[1])) for c in e.robot_grids]
        for k in range(12):
            m = np.zeros(shape, dtype=np.int32)
            if k % 3 == 1:  # one occupied footprint cell that lies inside the map, if any
                inside = [c for c in cells if c[0] < shape[0] and c[1] < shape[1]]
                if inside:
                    c = inside[int(erng.integers(0, len(inside)))]
                    m[c] = int(erng.integers(1, 256))
            elif k % 3 == 2:  # random clutter
                m = (erng.random(shape) < 0.08).astype(np.int32) * erng.integers(1, 256, shape).astype(np.int32)
            try:
                res = bool(e.is_collision(m))
            except IndexError:
                res = "IndexError"
            key = f"edge_{ci}_{k}"
            emaps[key] = m.astype(np.uint8)
            edge.append({"map": key, "map_grid_num": mg, "shape": list(shape), "result": res})
    out["is_collision_edge"] = edge
    maps.update(emaps)

    with open(os.path.join(OUT_DIR, "ref_pinned.json"), "w") as f:
        json.dump(out, f, indent=0, allow_nan=True)
    np.savez_compressed(os.path.join(OUT_DIR, "ref_maps.npz"), **maps)
    print("wrote", os.path.join(OUT_DIR, "ref_pinned.json"), "and ref_maps.npz")


if __name__ == "__main__":
    main()
