"""Child program of tests/test_gpu_timed_path.py: the EXACT path behind bench.py's metric, at
its full size, element for element against the C oracle (oracle/ffmp_oracle.c, bit-identical to
the NumPy oracle: tests/test_oracle_c.py).

The metric's workload is C3 — 32,768 envs of 256^2, 16 moving discs, 180 beams — stepped through
what bench.py's FFMPVec builds by default: the seamless frame ring (W = 8 physical slots, virtual
slot 8 a second mapping of slot 0; include/ffmp.h ffmp_ring_create) paired with the potential
plane, the partner relocation and the per-slot repair that run with a tuning, and newest-only
launches every step (the temporal stack of make_temporal_maps, /root/reference/src/train.py:474-486,
kept in place).  One instance, built the way bench.py builds it from a tuning, then:

  * slots 0 and 5 rebuilt with fresh pieces (ffmp_ring_rebuild: kept slots shared, replaced ones
    re-paired; the path the slot repair takes on a box with slow slots);
  * reset, and STEPS steps (>= W + 2, so every physical slot is written as the newest frame and
    then read as the older one, the alias slot included), each step through a different launch
    the autotune may choose: every one-launch flag set (FFMPVec.FUSED_FLAGS), then a two-launch
    step for EVERY raster shape candidate (FFMPVec.RASTER_SHAPES, incl. (4096, NT|XCD|TILE4), the
    shape behind the round-3 driver bench).  max_steps = 6 truncates and auto-resets every env inside a newest-only
    launch (both frames of every env written that step); collisions / goals reset single envs on
    other steps;
  * then (round 5) the step as bench.py's timed loop runs it: one HIP graph of a whole ring cycle
    (FFMPVec.capture) of the tuned two-launch step, of the tuned one-launch step and (float32) of the
    skewed step (raster i + env step i + 1 per launch), each replayed
    twice;
  * after the reset and after every step / replay, ALL envs are compared in 4,096-env slices: state_m (both
    frames, read through the ring view), the potential plane, the raster record, t, episode and the
    flags bit-exact; the float outputs within tests/parity_util.py's tolerances, and their exact
    mismatch counts reported.

The planes are compared on the GPU (the oracle's slice uploaded; one copy instead of a download
plus a host compare).  obs_format "u8f16" runs the same for the compact layout (bench.py's
`compact_layout` leg): uint8 frames == the oracle's 0/255 frames, binary16 potential == the
oracle's float32 plane rounded to nearest even (the rounding itself is pinned against numpy's in
tests/test_gpu_oracle_c.py::test_compact_c5_whole_on_one_gpu_in_slices).

Prints progress to stderr and ONE JSON summary line to stdout; exit status 0 iff parity holds.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import torch  # noqa: E402

from flow_field_based_motion_planner_amd import _abi  # noqa: E402
from flow_field_based_motion_planner_amd.config import preset  # noqa: E402
from flow_field_based_motion_planner_amd.vec_env import FFMPVec  # noqa: E402
from oracle.ffmp_oracle_c import COracleVecEnv  # noqa: E402
from tests.parity_util import compare, exact_report  # noqa: E402

SLICE = 4096
SMALL = ("state_g", "state_v", "state_t", "grad", "reward", "done", "is_goal", "collision", "truncated",
         "pose", "goal", "d0", "obst", "obst_r", "t", "episode", "record", "lidar")

# the bench's tuning as the driver's round-3 box chose it (BENCH_r03.json raster_autotune: two-launch
# step, newest-only raster (4096, NT|XCD|TILE4) = flags 37); the per-step plan below overrides the
# launch of every step anyway
TUNING = {"f32": {"shape": [4096, _abi.RASTER_NT | _abi.RASTER_XCD | _abi.RASTER_TILE4],
                  "shape_newest": [4096, _abi.RASTER_NT | _abi.RASTER_XCD | _abi.RASTER_TILE4],
                  "fused": False, "fused_flags": _abi.RASTER_NT | _abi.RASTER_XCD | _abi.RASTER_TILE4},
          "u8f16": {"shape": [65536, _abi.RASTER_NT | _abi.RASTER_TILE4 | _abi.RASTER_MID8],
                    "shape_newest": [65536, _abi.RASTER_NT | _abi.RASTER_TILE4 | _abi.RASTER_MID8],
                    "fused": False, "fused_flags": _abi.RASTER_NT | _abi.RASTER_TILE4 | _abi.RASTER_MID8}}


def launch_plan(fmt: str):
    """(fused, flags-or-shape) per step: EVERY launch the autotune may pick for this layout — each
    one-launch flag set (FUSED_FLAGS / COMPACT_FUSED_FLAGS), then a two-launch step for each raster
    shape candidate (RASTER_SHAPES / COMPACT_SHAPES) — so that the shape behind any bench line,
    including candidates added later, has run over the whole ring at full size."""
    if fmt == "f32":
        fused, two = FFMPVec.FUSED_FLAGS, FFMPVec.RASTER_SHAPES
    else:
        fused, two = FFMPVec.COMPACT_FUSED_FLAGS, FFMPVec.COMPACT_SHAPES
    return [(True, int(f)) for f in fused] + [(False, (int(c), int(f))) for c, f in two]


def small_snapshot(env, sl):
    d = {k: getattr(env, k)[sl].detach().cpu().numpy() for k in SMALL if getattr(env, k) is not None}
    d["lidar"] = d.get("lidar")
    return d


def check(env, ref, fmt: str, where: str, stats: dict) -> list:
    n, dev = env.num_envs, env.device
    problems = []
    osm, opot = ref.state_m, ref.potential
    for e0 in range(0, n, SLICE):
        sl = slice(e0, min(n, e0 + SLICE))
        # planes on the GPU, bit-exact
        o = torch.from_numpy(osm[sl]).to(dev)
        if fmt == "u8f16":
            o = o.to(torch.uint8)
        c = int((env.state_m[sl] != o).sum())
        if c:
            problems.append(f"{where} envs {e0}+ state_m: {c} cells differ")
        o = torch.from_numpy(opot[sl]).to(dev)
        if fmt == "u8f16":
            o = o.half()
            c = int((env.potential[sl].view(torch.int16) != o.view(torch.int16)).sum())
        else:
            c = int((env.potential[sl].view(torch.int32) != o.view(torch.int32)).sum())
        if c:
            problems.append(f"{where} envs {e0}+ potential: {c} cells not bit-identical")
        del o
        # everything else on the host, with tests/parity_util.py's tolerances (record, flags and
        # counters exact) — the planes were checked above, so compare() sees empty ones
        g = small_snapshot(env, sl)
        r = {k: (None if getattr(ref, k, None) is None else getattr(ref, k)[sl]) for k in SMALL}
        if not ref.cfg.n_beams:
            r["lidar"] = None
        empty = np.zeros(0, dtype=np.float32)
        g.update(state_m=empty, potential=None, flow=None, term_record=None, term_obs=None)
        r.update(state_m=empty, potential=None, flow=None, term_record=None, term_obs=None)
        problems += compare(g, r, f"{where} envs {e0}+")
        for k, v in exact_report(g, r).items():
            stats["not_bit_identical"][k] = stats["not_bit_identical"].get(k, 0) + v
        if len(problems) > 20:
            break
    return problems


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--obs-format", default="f32", choices=["f32", "u8f16"])
    ap.add_argument("--envs", type=int, default=32768)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--seed", type=int, default=33)
    ap.add_argument("--frame-window", type=int, default=8, help="bench.py's W (its automatic choice on a free GPU)")
    ap.add_argument("--out", default=None, help="also write the JSON summary to this file")
    args = ap.parse_args()
    fmt, n = args.obs_format, args.envs
    t0 = time.time()

    def log(msg):
        print(f"[{time.time() - t0:6.1f}s] {msg}", file=sys.stderr, flush=True)

    cfg = preset("C3", max_steps=6, seed=args.seed)
    env = FFMPVec(n, cfg, device="cuda:0", tuning=TUNING[fmt], obs_format=fmt, frame_window=args.frame_window)
    W = env.frame_window
    log(f"built {env!r}; ring {env.ring_meta}")
    if env.ring != "seamless" or W < 3:
        print(json.dumps({"ok": False, "why": f"not the bench's layout: ring={env.ring} W={W}"}))
        return 1
    # the repair's path: rebuild slots 0 (the alias slot's) and 5 with fresh pieces
    torch.cuda.synchronize()
    env._ring.rebuild((1 << 0) | (1 << 5), partner=env.potential)
    env._adopt_ring_tensor()
    plan = launch_plan(fmt)
    steps = max(len(plan), W + 2)
    plan = [plan[k % len(plan)] for k in range(steps)]
    ref = COracleVecEnv(cfg, n, threads=args.threads)
    stats = {"not_bit_identical": {}, "resets": 0, "collisions": 0, "goals": 0, "truncations": 0,
             "slots_written": [], "launches": []}
    env.reset()
    ref.reset()
    torch.cuda.synchronize()
    problems = check(env, ref, fmt, "reset", stats)
    rng = np.random.default_rng(args.seed)
    for k, (fused, how) in enumerate(plan):
        if problems:
            break
        env.fused = fused
        if fused:
            env.fused_flags = int(how)
        else:
            env.raster_shape_newest = tuple(how)
        a = rng.integers(0, 28, n)
        ep0 = int(env.episode.sum())
        env.step(torch.as_tensor(a, device="cuda:0"))
        ref.step(a)
        torch.cuda.synchronize()
        stats["slots_written"].append(env._slot_written(k))
        stats["launches"].append(["fused", int(how)] if fused else ["two", list(how)])
        stats["resets"] += int(env.episode.sum()) - ep0
        stats["collisions"] += int(env.collision.sum())
        stats["goals"] += int(env.is_goal.sum())
        stats["truncations"] += int(env.truncated.sum())
        problems += check(env, ref, fmt, f"step {k} ({stats['launches'][-1]})", stats)
        log(f"step {k} {stats['launches'][-1]}: slot {stats['slots_written'][-1]}, "
            f"{len(problems)} problems, {stats['resets']} resets so far")
    # bench.py's timed loop replays one HIP graph of a whole ring cycle (FFMPVec.capture, --graph):
    # the tuned two-launch step and the tuned one-launch step, each captured from where the eager
    # plan left the ring and replayed twice, all envs checked after every replay
    # (and the skewed graph, ffmp_step_skewed — one launch per step — which bench.py keeps where it
    # is faster: float32 frames only)
    from flow_field_based_motion_planner_amd.vec_env import StepGraph
    modes = [(False, False), (True, False)]
    if StepGraph.skew_supported(env, env.graph_period()):
        modes.append((False, True))
    for fused, skewed in modes:
        if problems:
            break
        env.fused = fused
        if fused:
            env.fused_flags = int(TUNING[fmt]["fused_flags"])
        else:
            env.raster_shape_newest = tuple(TUNING[fmt]["shape_newest"])
        g = env.capture(skewed=skewed)
        for r in range(2):
            if problems:
                break
            acts = rng.integers(0, 28, (g.steps, n))
            ep0 = int(env.episode.sum())
            g.replay(torch.as_tensor(acts, device="cuda:0"))
            for a in acts:
                ref.step(a)
            torch.cuda.synchronize()
            how = (["graph-fused", int(env.fused_flags)] if fused else
                   ["graph-skewed" if skewed else "graph-two", list(env.raster_shape_newest)])
            stats["launches"].append(how + [g.steps])
            stats["resets"] += int(env.episode.sum()) - ep0
            problems += check(env, ref, fmt, f"graph replay {r} ({how})", stats)
            log(f"graph replay {r} {how} x {g.steps} steps: {len(problems)} problems, {stats['resets']} resets so far")
        del g
    env.check_errors()
    out = {"ok": not problems, "obs_format": fmt, "n_envs": n, "frame_window": W, "ring": env.ring,
           "steps": len(plan), "problems": problems[:20], "ring_meta": env._ring.info(), **stats,
           "tuning": TUNING[fmt], "seconds": round(time.time() - t0, 1)}
    print(json.dumps(out), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)
    return 0 if not problems else 1


if __name__ == "__main__":
    sys.exit(main())
