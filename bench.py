#!/usr/bin/env python3
"""Throughput benchmark of the batched FFMP step on MI355X (driver contract).

One "step" = one FFMPVec step of every env this rank owns: the env kernel
(integrate, obstacles, lidar, collision/reward/done, auto-reset) + the raster
kernel (the new float32 frame of the state_m temporal stack — both frames when
the frame window wraps or an env resets — and the float32 potential plane).
Actions for every timed step are pre-generated on the device (inputs resident
in HBM before the timed region).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config C3]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

With --gpus N > 1 and no torchrun environment (WORLD_SIZE unset), this process starts the N rank
processes itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT in each
child's environment) before anything touches the GPU, waits for them and exits with the first
non-zero status; every rank checks that its process group has exactly N members.

N=1 workload: BASELINE config C3 (32,768 envs, 256x256 grid, 16 moving discs,
180-beam lidar) — the largest single-GPU config and the one the north-star
target (256x256, 32k envs) is quoted on.  Every run has two legs:

  weak    C3 per rank (32,768 envs on each of the N GPUs) — the line's `value`
  strong  C4: 65,536 envs split over the N ranks (`strong`; --strong-config none skips)

so the driver's 1/2/4/8-GPU runs yield both scaling curves.  No data-path collective
(env shards; one max-reduce of the timings).  --config C4/C5 makes the main leg
split its total over the ranks instead.  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "env-steps/sec (batched gym_ffmp) at 1/2/4/8 MI355X; HBM-roofline %"
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md: 8.0 TB/s)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--config", default="C3", choices=["C2", "C3", "C4", "C5"])
    p.add_argument("--envs", type=int, default=0, help="override envs per rank")
    p.add_argument("--env-offset", type=int, default=None,
                   help="global index of this rank's first env (default rank x envs); e.g. --config C4 --envs 8192 "
                        "--env-offset 57344 runs the 8-GPU strong leg's rank-7 shard on one GPU")
    p.add_argument("--no-potential", action="store_true")
    p.add_argument("--flow", action="store_true", help="also raster the BEV motion-flow planes (not a BASELINE config)")
    p.add_argument("--cpu-seconds", type=float, default=15.0, help="CPU-baseline time budget (0 = skip)")
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="host threads of the C-oracle CPU baseline (SURVEY 8d (ii)); 0 = every CPU this process "
                        "may run on (affinity mask, capped by the cgroup CPU quota)")
    p.add_argument("--strong-config", default="C4", choices=["none", "C4", "C5"],
                   help="second leg: this preset's TOTAL env count split over the ranks (strong scaling)")
    p.add_argument("--strong-steps", type=int, default=None, help="timed steps of the strong leg (default --steps)")
    p.add_argument("--dump-launches", action="store_true", help="print every timed raster launch (ms) to stderr")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--pipeline", type=int, default=None, help="env/raster pipeline slices (default: automatic)")
    p.add_argument("--frame-window", type=int, default=None,
                   help="frames per env kept in HBM (2 = contiguous (N,2,G,G) rewritten every step; default auto)")
    p.add_argument("--ring", default="auto", choices=["auto", "seamless", "wrap"],
                   help="frame ring with frame_window > 2: seamless (VMM alias, never wraps) or wrap")
    p.add_argument("--fused", default="auto", choices=["auto", "on", "off"],
                   help="one-launch step (ffmp_step_fused) on/off, or auto: the instance's autotune decides")
    p.add_argument("--graph", default="on", choices=["off", "on"],
                   help="on (default): the timed steps run as replays of one HIP graph of graph_period() whole "
                        "steps (FFMPVec.capture: the same env + raster launches as step(), no launch gaps or host "
                        "work between them); the roofline's kernel is then the replayed step graph (its env and "
                        "raster kernels, their bytes).  off: one step() call per step")
    p.add_argument("--graph-skew", default="auto", choices=["auto", "on", "off"],
                   help="with --graph on: replay graphs whose steps are ONE launch each (the raster of step i + the "
                        "env step of step i + 1, ffmp_step_skewed; open loop: actions known a step ahead) — auto: time both graphs (8 alternating replays "
                        "each, untimed) and keep the faster; on / off: force")
    p.add_argument("--closed-loop", type=int, default=1,
                   help="1 (default): after the open-loop timing, time the main leg closed-loop too (each step's "
                        "actions computed on the device from the previous observation: `closed_loop`); 0: skip")
    p.add_argument("--save-tuning", default=None, help="write the instance's launch choices (JSON) here")
    p.add_argument("--tuning", default=None,
                   help="launch choices from --save-tuning instead of the autotune (profiling runs: only timed "
                        "launches of the dominant kernel in the trace)")
    p.add_argument("--obs-format", default="f32", choices=["f32", "u8f16"],
                   help="f32: the reference consumer layout (state_m float32, the bench metric); u8f16: the "
                        "compact layout (uint8 frames, float16 potential) for consumers that convert on load")
    p.add_argument("--compact-steps", type=int, default=100,
                   help="N=1 f32 runs: also time this many steps of the same workload in the compact layout "
                        "(obs_format=u8f16), reported as `compact_layout` beside the metric (0 = skip)")
    p.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                   help="nccl (= RCCL on ROCm) for real runs; gloo only to rehearse several ranks on one GPU")
    return p.parse_args()


def _time_oracle(env, n, seconds: float, seed: int):
    """Step an oracle env on random actions for about `seconds`; (env-steps, seconds)."""
    import numpy as np
    rng = np.random.default_rng(seed)
    env.reset()
    env.step(rng.integers(0, 28, n))  # warm
    steps, t0 = 0, time.perf_counter()
    while True:
        env.step(rng.integers(0, 28, n))
        steps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            return n * steps, el


def _cgroup_cpus():
    """CPUs the cgroup (v2 cpu.max, else v1 cfs quota) lets this process use, or None if unlimited."""
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(path).read().split()[:2]
            if q != "max":
                return float(q) / float(per)
        except (OSError, ValueError):
            pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0:
            return q / per
    except (OSError, ValueError):
        pass
    return None


def host_cpus() -> dict:
    """What the host offers this process: os.cpu_count() (the whole machine), the affinity mask,
    the cgroup quota; `usable` = the mask capped by the quota (what the CPU baseline runs on)."""
    try:
        allowed = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        allowed = os.cpu_count() or 1
    quota = _cgroup_cpus()
    usable = max(1, min(allowed, int(quota)) if quota else allowed)
    return {"cpu_count": os.cpu_count(), "allowed_cpus": allowed, "cgroup_cpus": quota, "usable": usable}


def cpu_baseline(cfg, seconds: float, threads: int):
    """The C restatement of the oracle (oracle/ffmp_oracle.c, bit-identical to the NumPy oracle:
    tests/test_oracle_c.py) stepping a bounded sample of the same workload on every CPU this
    process may use (threads = 0: the affinity mask capped by the cgroup quota; one env per thread
    at a time, OpenMP over envs) — SURVEY 8(d)(ii) — plus the same on 16 threads (round 2's
    figure), on one thread (8(d)(i)) and the NumPy oracle on one thread (the round-1 baseline)."""
    from oracle.ffmp_oracle import OracleVecEnv
    from oracle.ffmp_oracle_c import COracleVecEnv, load
    cpus = host_cpus()
    threads = cpus["usable"] if threads <= 0 else max(1, min(threads, cpus["allowed_cpus"]))
    # single-threaded legs first: the OpenMP pool's idle threads spin for a while after a region
    k2, el2 = _time_oracle(OracleVecEnv(cfg, 4), 4, seconds / 3, 2)
    try:
        k1, el1 = _time_oracle(COracleVecEnv(cfg, 4, threads=1), 4, seconds / 3, 1)
        n = 4 * threads
        k, el = _time_oracle(COracleVecEnv(cfg, n, threads=threads), n, seconds, 0)
        k16 = el16 = None
        if threads != 16:
            k16, el16 = _time_oracle(COracleVecEnv(cfg, 64, threads=16), 64, seconds / 3, 4)
    except (OSError, RuntimeError) as exc:  # C oracle not built / not loadable here: the NumPy leg only
        k3, el3 = _time_oracle(OracleVecEnv(cfg, 4), 4, seconds, 2)
        return {"value": k3 / el3, "unit": "env-steps/s", "cores": 1, "kind": "port", "cpu_model": _cpu_model(),
                "host_cpus": cpus,
                "sample": f"4 envs x {k3 // 4} steps ({el3:.1f} s), NumPy oracle, 1 thread (C oracle unavailable: {exc})"}
    from flow_field_based_motion_planner_amd.config import preset
    c1 = preset("C1")  # BASELINE configs[0]: one env, 64x64, 4 static discs, the reference's CPU case
    k3, el3 = _time_oracle(OracleVecEnv(c1, 1), 1, 2.0, 3)
    return {"value": k / el, "unit": "env-steps/s", "cores": threads, "kind": "port", "cpu_model": _cpu_model(),
            "host_cpus": cpus,
            "sample": f"{n} envs x {k // n} steps of the same config ({el:.1f} s), C oracle "
                      f"(oracle/ffmp_oracle.c, {os.path.basename(load().path)}), {threads} threads "
                      f"(every usable CPU: affinity {cpus['allowed_cpus']}, cgroup quota {cpus['cgroup_cpus']})",
            "threads16": ({"value": k / el, "cores": 16, "sample": "the main figure (16 usable CPUs)"} if k16 is None else
                          {"value": k16 / el16, "cores": 16, "sample": f"64 envs x {k16 // 64} steps ({el16:.1f} s), "
                                                                         "16 threads"}),
            "one_core": {"value": k1 / el1, "cores": 1, "sample": f"4 envs x {k1 // 4} steps ({el1:.1f} s), 1 thread"},
            "numpy_one_core": {"value": k2 / el2, "cores": 1,
                               "sample": f"4 envs x {k2 // 4} steps ({el2:.1f} s), NumPy oracle OracleVecEnv, "
                                         f"1 thread"},
            "c1_numpy_single_env": {"value": k3 / el3, "cores": 1,
                                    "sample": f"C1 (1 env, 64x64, 4 static discs, no lidar): {k3} steps "
                                              f"({el3:.1f} s), NumPy oracle, 1 thread"}}


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def load_traffic(workload: str, n_envs: int, window: int, ring: str, fused: bool, obs_format: str = "f32",
                 graph_steps: int = 0, graph_skewed: bool = False):
    """(HBM bytes per timed launch, the profile file it came from) from the committed rocprofv3 PMC
    summary, if one matches this launch — the raster (or one-launch step) kernel, or with
    graph_steps > 0 one replay of that many whole steps; (None, None) otherwise."""
    b = _load_traffic(workload, n_envs, window, ring, fused, obs_format, graph_steps, graph_skewed)
    return b if b is not None else (None, None)


def _load_traffic(workload, n_envs, window, ring, fused, obs_format, graph_steps=0, graph_skewed=False):
    label = f"{workload}{'' if obs_format == 'f32' else '_' + obs_format}"
    gsfx = "_graph" if graph_steps else ""
    path = os.path.join(ROOT, "profiles", f"pmc_traffic_{label}{'_fused' if fused else ''}{gsfx}.json")
    if not os.path.exists(path):  # the one-launch and two-launch steps are profiled separately
        path = os.path.join(ROOT, "profiles", f"pmc_traffic_{label}{gsfx}.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            d = json.load(f)
        if int(d.get("n_envs", -1)) != n_envs or int(d.get("frame_window", 2)) != window \
                or d.get("ring", "wrap" if window > 2 else "contiguous") != ring or bool(d.get("fused", False)) != fused \
                or d.get("obs_format", "f32") != obs_format or int(d.get("graph_steps", 0)) != int(graph_steps) \
                or bool(d.get("skewed", False)) != bool(graph_skewed and graph_steps):
            return None
        key = "step_graph_hbm_bytes_per_replay" if graph_steps else "raster_hbm_bytes_per_launch"
        return float(d[key]), os.path.relpath(path, ROOT)
    except Exception:  # noqa: BLE001
        return None


def time_compact(FFMPVec, name, cfg, n, dev, steps, warmup, seed):
    """The same workload in the compact layout (uint8 frames, float16 potential; include/ffmp.h
    FFMP_OBS_U8F16) on a fresh instance: whole-step rate and its raster's rate against HBM peak.
    Not the metric (the reference consumer layout is float32), reported beside it."""
    import torch
    from flow_field_based_motion_planner_amd.config import bytes_per_env_step
    env = FFMPVec(n, cfg, device=dev, obs_format="u8f16")
    gen = torch.Generator(device=dev).manual_seed(2000 + seed)
    actions = torch.randint(0, 28, (warmup + steps, n), device=dev, dtype=torch.int64, generator=gen)
    env.reset()
    for w in range(warmup):
        env.step(actions[w])
    torch.cuda.synchronize()
    ep0 = int(env.episode.sum())
    ev, t = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)), []
    t0 = time.perf_counter()
    ev[0].record()
    for k in range(steps):
        env.step(actions[warmup + k], timing=t)
    ev[1].record()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    resets = int(env.episode.sum()) - ep0
    ms = [r[0].elapsed_time(r[1]) for r in t]
    n_full = sum(1 for r in t if r[4])
    byt = sum(r[3] for r in t) + resets * (len(t) - n_full) / len(t) * cfg.grid * cfg.grid
    ach = byt / (sum(ms) * 1e-3) / 1e9
    b = bytes_per_env_step(cfg, potential=True, window=env.frame_window, seamless=env.ring == "seamless",
                           obs_format="u8f16")
    out = {"obs_format": "u8f16", "value": n * steps / el, "unit": "env-steps/s", "steps": steps,
           "ms_per_step": el * 1e3 / steps, "step_ms_events": ev[0].elapsed_time(ev[1]) / steps,
           "kernel": "step_raster_kernel" if env.fused else "raster_kernel", "kernel_ms": sum(ms) / len(ms),
           "achieved_gbs": ach, "frac": ach / PEAK_HBM_GBS, "bytes_per_env_step": b["total"],
           "frame_window": env.frame_window, "ring": env.ring, "fused": bool(env.fused),
           "shape": (env.placement or {}).get("shape_newest"),
           "ring_pairing": {k: (env.ring_meta or {}).get(k) for k in ("pieces", "pair_probes", "pair_gbs_min",
                                                                        "pair_gbs_max", "rebuilds", "reverts")}}
    env.close()
    return out


def time_compact_child(name, steps, seed):
    """The compact-layout leg in a child process of its own (bench.py --obs-format u8f16), as a user
    running that layout would: this process has parked its float32 rings' pieces (never unmapped,
    DESIGN §4), and a compact ring built here would draw them first.  None if the child fails."""
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), "--config", name, "--obs-format", "u8f16", "--strong-config",
           "none", "--cpu-seconds", "0", "--compact-steps", "0", "--steps", str(steps), "--warmup", "10",
           "--seed", str(seed)]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
    except subprocess.TimeoutExpired:
        print("warning: compact-layout child timed out", file=sys.stderr)
        return None
    line = next((ln for ln in reversed(r.stdout.splitlines()) if ln.startswith("{")), None)
    if r.returncode != 0 or line is None:
        print(f"warning: compact-layout child failed (rc {r.returncode}): {r.stderr[-2000:]}", file=sys.stderr)
        return None
    d = json.loads(line)
    rl, a = d["roofline"], d.get("raster_autotune", {})
    ring = a.get("ring") or {}
    return {"obs_format": "u8f16", "value": d["value"], "unit": "env-steps/s", "steps": d["steps"],
            "ms_per_step": d["ms_per_step"], "step_ms_events": d["step_ms_events"], "kernel": rl["kernel"],
            "kernel_ms": rl["kernel_ms"], "achieved_gbs": rl["achieved"], "frac": rl["frac"],
            "algorithmic_bytes_per_launch": rl["algorithmic_bytes_per_launch"], "traffic": rl.get("traffic"),
            "frame_window": d["config"]["frame_window"], "ring": d["config"]["ring"], "fused": d["config"]["fused"],
            "shape": a.get("shape_newest"), "construct_s": d.get("construct_s"), "hbm_bytes": d.get("hbm_bytes"),
            "ring_pairing": {k: ring.get(k) for k in ("pieces", "pair_probes", "pair_gbs_min", "pair_gbs_max",
                                                      "partner_tries", "rebuilds", "reverts", "repair",
                                                      "pool_released_bytes")},
            # the child's launch decisions, for audit: every raster-shape candidate's GB/s, the
            # one-launch vs two-launch step times (autotune and post-repair recheck), the flags kept
            "autotune": {k: a.get(k) for k in ("shape", "shape_newest", "gbs", "candidates", "fused")},
            "hbm_in_use_bytes": d.get("hbm_in_use_bytes"),
            "process": "a child process of its own (bench.py --obs-format u8f16)"}


def _gather_floats(vals, world, dev, backend):
    """Every rank's `vals` (list of floats) -> (world, len) list of lists; one collective."""
    import torch
    import torch.distributed as dist
    t = torch.tensor(vals, dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    if world == 1:
        return [t.tolist()]
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [o.tolist() for o in out]


# What every rank reports after its timed region (one all_gather, never inside it): enough to
# explain a max-over-ranks line — which rank was slow, and whether its kernel, its launch choice
# (one- or two-launch step, raster shape) or its HBM pairing (ring slot times, the weakest accepted
# piece pairing) made it so.  NaN = not applicable (no seamless ring, no repair timing).
RANK_FIELDS = ("elapsed_s", "construct_s", "n_envs", "kernel_ms", "frac", "fused", "shape_cells", "shape_flags",
               "slot_ms_min", "slot_ms_max", "pair_gbs_min")


def rank_record(el_local: float, construct_s: float, n: int, kernel_ms: float, frac: float, env) -> list:
    """This rank's RANK_FIELDS values (floats) from its timed loop and its FFMPVec."""
    nan = float("nan")
    pl = getattr(env, "placement", None) or {}
    fused = bool(getattr(env, "fused", False))
    sh = pl.get("shape_newest") or pl.get("shape") or {}
    cells = nan if fused else float(sh.get("cells_per_block", nan))
    flags = float((pl.get("fused") or {}).get("flags", nan)) if fused else float(sh.get("flags", nan))
    meta = getattr(env, "ring_meta", None) or {}
    slots = next((h["slot_ms"] for h in reversed(meta.get("repair") or []) if "slot_ms" in h and not h.get("reverted")),
                 None)
    return [float(el_local), float(construct_s), float(n), float(kernel_ms), float(frac), float(fused), cells, flags,
            float(min(slots)) if slots else nan, float(max(slots)) if slots else nan,
            float(meta.get("pair_gbs_min", nan) or nan)]


def per_rank_table(rows) -> dict:
    """Gathered rank records (rank order) -> {field: [value of rank 0, rank 1, ...]} (NaN -> None)."""
    def clean(v):
        return None if v != v else (int(v) if v == int(v) and abs(v) < 2 ** 53 else round(v, 5))
    return {f: [clean(r[i]) for r in rows] for i, f in enumerate(RANK_FIELDS)}


def run_leg(args, name, cfg, n, offset, K, W, dev, world, rank, strong, main_leg):
    """Build one FFMPVec shard (timed: construct_s), W warm-up + K timed steps between barriers and
    synchronizes, max over ranks; the dominant kernel's launches timed with HIP events on the
    launch stream.  Returns (summary dict, env)."""
    import torch
    import torch.distributed as dist
    from flow_field_based_motion_planner_amd.config import bytes_per_env_step
    from flow_field_based_motion_planner_amd.vec_env import FFMPVec
    fb = 4 if args.obs_format == "f32" else 1
    # the actions first: the first use of torch's random kernels loads their code (a GPU-idle gap),
    # and after such a gap the raster runs slow for about one ring cycle while the GPU warms up again
    # (profiles/r03b_transient*.txt) — here that gap falls before construction, not before the warm-up
    gen = torch.Generator(device=dev).manual_seed(1000 + rank + (0 if main_leg else 5000))
    actions = torch.randint(0, 28, (W + K, n), device=dev, dtype=torch.int64, generator=gen)
    torch.cuda.synchronize(dev)
    t_c = time.perf_counter()
    env = FFMPVec(n, cfg, device=dev, env_offset=offset, potential=not args.no_potential, pipeline=args.pipeline,
                  frame_window=args.frame_window, seamless={"auto": None, "seamless": True, "wrap": False}[args.ring],
                  fused={"auto": None, "on": True, "off": False}[args.fused],
                  tuning=json.load(open(args.tuning)) if (args.tuning and main_leg) else None,
                  obs_format=args.obs_format)
    torch.cuda.synchronize(dev)
    construct_s = time.perf_counter() - t_c
    if args.save_tuning and rank == 0 and main_leg:
        with open(args.save_tuning, "w") as f:
            json.dump(env.tuning(), f)
    free, total = torch.cuda.mem_get_info(dev)
    # the torch kernel the loop's bookkeeping uses (episode.sum) is loaded now: its first call loads
    # its code with the GPU idle, and after such a gap the raster runs slow for about one ring cycle
    # (profiles/r03b_transient_loop.txt) — it must not fall between the warm-up
    # and the timed steps
    int(env.episode.sum())
    env.reset()
    for w in range(W):
        env.step(actions[w])
    # one event pair around the timed loop (per-step pairs add a stream marker between launches,
    # ~10 % of a C2 step); the dominant kernel keeps its per-launch pairs (roofline.achieved)
    ev_loop = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    raster_ev = []
    graph, graph_error, skew_trial = None, None, None
    if args.graph == "on" and K >= env.graph_period() and env.pipeline_slices == 1:
        # one graph of graph_period() whole steps, captured and replayed once (untimed, the warm-up's
        # actions) before the timed region; the timed steps are K // period replays + K % period steps
        try:
            from flow_field_based_motion_planner_amd.vec_env import StepGraph
            per0 = env.graph_period()
            can_skew = StepGraph.skew_supported(env, per0) and args.graph_skew != "off"
            graph = env.capture(skewed=bool(can_skew and args.graph_skew == "on"))
            if can_skew and args.graph_skew == "auto":
                # the skewed graph (one launch per step) against the two-launch one: 8 alternating
                # replays each after one warm replay, the faster (median) kept (C2: the env waves hide
                # beside the raster; C3: 2,048 env blocks dispatched first delay the raster's stores).
                # Open loop only: a skewed step needs step i + 1's actions before step i's observation
                gs = env.capture(skewed=True)
                ms = {False: [], True: []}
                for g in (graph, gs):
                    g.replay(actions[:per0])
                for _ in range(8):
                    for key, g in ((False, graph), (True, gs)):
                        a0, a1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        a0.record()
                        g.replay(actions[:per0])
                        a1.record()
                        torch.cuda.synchronize()
                        ms[key].append(a0.elapsed_time(a1))
                med = {key: sorted(v)[len(v) // 2] for key, v in ms.items()}
                chosen = med[True] < 0.995 * med[False]
                skew_trial = {"chosen": chosen, "serial_replay_ms": [round(v, 4) for v in ms[False]],
                              "skewed_replay_ms": [round(v, 4) for v in ms[True]]}
                if chosen:
                    graph = gs
        except Exception as exc:  # noqa: BLE001 — a box whose runtime refuses the capture: step() instead
            print(f"warning: HIP graph capture failed, timing step() calls instead: {exc}", file=sys.stderr)
            graph_error = str(exc)[:300]
            graph = None
    graph_rem = None
    if graph is not None:
        per = graph.steps
        rem = K % per
        fulls = [env.frame_window == 2 or (env.ring != "seamless" and i == per - 1) for i in range(per)]
        graph_bytes = sum(env._raster_bytes(n, f) + env._state_bytes(n) for f in fulls)
        # the last K % period steps: a graph of their own, captured from the same position (each
        # timed step is a replayed step); warmed once like the full one, then the ring is stepped back
        # to the start (untimed)
        graph.replay(actions[:per])
        if rem:
            graph_rem = env.capture(rem, skewed=bool(graph.skewed and rem % 2 == 0))
            rem_bytes = sum(env._raster_bytes(n, f) + env._state_bytes(n) for f in fulls[:rem])
            graph_rem.replay(actions[:rem])
            for k in range(rem, per):
                env.step(actions[k])
        # The graph warm-ups and the skew trial above stepped every env ~150-190 steps past the warm-up.
        # Every env starts its first episode at the same reset, so the ~85 % that survive max_steps (200)
        # random-action steps truncate and reset on the SAME step. After the 8-round skew trial that step
        # fell inside the 20 timed steps: 27,807 resets in the window against 611 (profiles/r06g_*,
        # r06h_*), 13.4-13.7 vs 13.9-14.0 M. A long run pays that step once per 200. Restart the episodes
        # instead: reset, then the W warm-up steps again, which also brings the ring back to the position
        # the graphs were captured at. The timed steps then start from a fresh reset plus warm-up, as
        # they did before the trials existed.
        env.reset()
        for w in range(W):
            env.step(actions[w])
        # re-warm: the captures above (torch.cuda.graph synchronizes, collects garbage and empties the
        # cache) leave the GPU idle for a while, and after an idle gap the first few ms of steps run slow
        # (profiles/r03b_transient*.txt) — at the 8-GPU strong leg's 0.6-ms steps the driver's 20 timed
        # steps fell to 0.80 of the roofline from 0.90 at 200 (profiles/r06a_bench_c4_8192_*.json).  Replay
        # the graph for >= 30 ms of GPU work (untimed, the warm-up's actions) right before the timed region.
        t_one = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t_one[0].record()
        graph.replay(actions[:per])
        t_one[1].record()
        torch.cuda.synchronize()
        for _ in range(max(1, int(30.0 / max(t_one[0].elapsed_time(t_one[1]), 1e-3)))):
            graph.replay(actions[:per])
        torch.cuda.synchronize()
    ep0_t = env.episode.sum()  # read after the loop: no host round trip between the sync and the loop
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev_loop[0].record()
    if graph is None:
        for k in range(K):
            env.step(actions[W + k], timing=raster_ev)
    else:
        for r in range(K // per):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            graph.replay(actions[W + r * per:W + (r + 1) * per])
            e1.record()
            raster_ev.append((e0, e1, n, graph_bytes, False))
        if graph_rem is not None:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            graph_rem.replay(actions[W + K - rem:W + K])
            e1.record()
            raster_ev.append((e0, e1, n, rem_bytes, False))
    ev_loop[1].record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el_local = time.perf_counter() - t0
    env.check_errors()
    resets = int(env.episode.sum()) - int(ep0_t)  # auto-resets in the timed steps

    # the dominant kernel — the raster, or with the one-launch step the fused env-step + raster
    # kernel: HIP events around every launch on the launch stream; algorithmic bytes per launch
    # from the frame-window schedule (full launches write both frames; the fused kernel adds the
    # env step's state bytes), plus the older frame of every env reset during a newest-only
    # launch (resets spread evenly over launches)
    r_ms = [r[0].elapsed_time(r[1]) for r in raster_ev]
    if args.dump_launches and main_leg:
        print("raster ms per launch:", " ".join(f"{x:.3f}" for x in r_ms), file=sys.stderr, flush=True)
    n_full = sum(1 for r in raster_ev if r[4])
    G2 = cfg.grid * cfg.grid
    # resets spread evenly over the timed launches
    if graph is None:
        r_bytes = sum(r[3] for r in raster_ev) + resets * (len(raster_ev) - n_full) / (K * env.pipeline_slices) * fb * G2
    else:  # the replayed steps' newest-only rasters write an older frame for each env they reset
        new_frac = sum(1 for f in fulls if not f) / per
        r_bytes = sum(r[3] for r in raster_ev) + resets * new_frac * fb * G2
    b = bytes_per_env_step(cfg, potential=not args.no_potential, window=env.frame_window,
                           seamless=env.ring == "seamless", obs_format=args.obs_format)
    achieved = r_bytes / (sum(r_ms) * 1e-3) / 1e9
    # one all_gather of every rank's record after the timed region (the max-reduce of the timings
    # is its first column)
    # the dominant kernel's mean launch: per step's raster (or one-launch step), or with graph
    # replays per full-period replay (a shorter remainder replay counts in `achieved` only)
    kernel_ms = (sum(r_ms[:K // per]) / (K // per)) if graph is not None else sum(r_ms) / len(r_ms)
    per_rank = _gather_floats(rank_record(el_local, construct_s, n, kernel_ms, achieved / PEAK_HBM_GBS, env),
                              world, dev, args.dist_backend)
    closed = None
    if main_leg and args.closed_loop and env.pipeline_slices == 1:
        closed = closed_loop_leg(env, K, W, world, dev, args.dist_backend, b["total"], el_local * 1e3 / K)
    el = max(r[0] for r in per_rank)  # == the max-reduce over ranks
    n_total = int(sum(r[2] for r in per_rank))
    out = {
        "workload": name, "n_envs_total": n_total, "n_envs_per_gpu": n, "scaling": "strong" if strong else "weak",
        "value": n_total * K / el, "ms_per_step": el * 1e3 / K, "steps": K, "warmup": W,
        "per_rank_ms_per_step": [round(r[0] * 1e3 / K, 4) for r in per_rank],
        "per_rank_construct_s": [round(r[1], 2) for r in per_rank],
        "per_rank": per_rank_table(per_rank),
        "construct_s": round(construct_s, 2), "hbm_bytes": env.hbm_bytes(),
        "hbm_in_use_bytes": int(total - free), "hbm_total_bytes": int(total),
        "pool_released_bytes": getattr(env, "pool_released_bytes", 0),
        "frame_window": env.frame_window, "ring": env.ring, "fused": bool(env.fused),
        "graph": ({"steps_per_replay": per, "replays": K // per, "remainder_steps": rem,
                   "skewed": bool(graph.skewed), "skew_trial": skew_trial} if graph is not None else
                  {"error": graph_error} if graph_error else None),
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": achieved / PEAK_HBM_GBS,
                     "kernel": ("step graph (%s x %d steps)" % ("step_raster_kernel" if env.fused else
                                                                 "skew_kernel: raster i + env step i+1" if graph.skewed
                                                                 else "env_kernel + raster_kernel", per)
                                if graph is not None else "step_raster_kernel" if env.fused else "raster_kernel"),
                     # with graph replays: per replay of `per` steps (the full-period replays; a shorter
                     # remainder replay counts in `achieved` only)
                     "kernel_ms": kernel_ms,
                     "algorithmic_bytes_per_launch": (r_bytes * per / K) if graph is not None else
                                                     r_bytes / len(raster_ev),
                     "launches_per_step": env.pipeline_slices, "timed_launches": len(r_ms),
                     "full_launches": n_full, "timed_resets": resets},
        "raster_ms_per_step": sum(r_ms) / K,
        "step_ms_events": ev_loop[0].elapsed_time(ev_loop[1]) / K,
        "pipeline_slices": env.pipeline_slices,
        "raster_autotune": env.placement,
        "hbm_roofline_pct_whole_step": 100.0 * (b["total"] * n_total * K / el / 1e9) / (PEAK_HBM_GBS * world),
        "per_launch_envs": raster_ev[0][2],
        "closed_loop": closed,
    }
    if closed is not None:
        for k in ("step_graph", "step_plain", "policy_graph"):
            closed[k]["vs_open_loop"] = closed[k]["value"] / out["value"]
    return out, env


def closed_loop_leg(env, K: int, warm: int, world: int, dev, backend: str, step_bytes: float,
                    step_ms: float) -> dict:
    """Closed loop (src/train.py:572-577, 665-682: each action is chosen from the previous
    observation, never known a step ahead): step k + 1's actions come from step k's observation on
    the device (FFMPVec.policy_reactive, include/ffmp.h ffmp_policy_reactive: reads state_g and the
    newest frame) inside the timed region.  Three forms, K steps each, max over ranks:
      step_graph   the per-step API — policy_reactive into action_buffer, then step() replaying a
                   single-step HIP graph (FFMPVec.use_graphs);
      step_plain   the same loop with plain launches;
      policy_graph the policy captured inside a graph of graph_period() steps (capture(policy=...)),
                   replayed with no host work between steps (the K % period rest: step_graph steps).
    Each form's timed region follows >= 30 ms of its own untimed steps (the GPU-idle transient)."""
    import math
    import torch
    import torch.distributed as dist
    n = env.num_envs
    warm = max(warm, int(math.ceil(30.0 / max(step_ms, 1e-3))))
    out = {"policy": "ffmp_policy_reactive (scripted controller; reads state_g and the newest frame)",
           "steps": K}

    def timed(body):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        body()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        return time.perf_counter() - t0

    def step_loop(k):
        for _ in range(k):
            env.step(env.policy_reactive(out=env.action_buffer))

    env.use_graphs(True)
    step_loop(env.graph_period() + 1)  # every ring position's graph captured ...
    step_loop(warm)                     # ... then warm
    el = {"step_graph": timed(lambda: step_loop(K))}
    env.use_graphs(False)
    step_loop(warm)
    el["step_plain"] = timed(lambda: step_loop(K))
    env.use_graphs(True)
    per = env.graph_period()
    pg = env.capture(policy="reactive")
    for _ in range(max(1, -(-warm // pg.steps))):
        pg.replay()
    rem = K % pg.steps
    torch.cuda.synchronize()

    def graph_loop():
        for _ in range(K // pg.steps):
            pg.replay()
        step_loop(rem)
    el["policy_graph"] = timed(graph_loop)
    env.use_graphs(False)
    keys = ("step_graph", "step_plain", "policy_graph")
    rows = _gather_floats([el[k] for k in keys], world, dev, backend)
    for i, k in enumerate(keys):
        t = max(r[i] for r in rows)
        rate = n * world * K / t  # equal shards: every rank steps n envs
        out[k] = {"value": rate, "unit": "env-steps/s", "ms_per_step": t * 1e3 / K,
                  "hbm_roofline_pct_whole_step": 100.0 * step_bytes * rate / 1e9 / (PEAK_HBM_GBS * world)}
    out["policy_graph"]["steps_per_replay"] = pg.steps
    out["graph_period"] = per
    env.check_errors()
    return out


def _release(env):
    import gc
    import torch
    env.close()
    del env
    gc.collect()
    torch.cuda.empty_cache()


def _leg_size(name, args, world, dev):
    """(envs per rank, strong?) for preset `name`: strong-scaling presets (C4/C5) split their total
    over the ranks; a shard that would not fit one GPU's HBM falls back to the preset's per-GPU
    share (weak)."""
    import torch
    from flow_field_based_motion_planner_amd.config import PRESETS, preset
    pr = PRESETS[name]
    cfg = preset(name, seed=args.seed, flow=args.flow)
    strong = pr["gpus"] > 1
    n = args.envs or (pr["n_envs"] // world if strong else pr["n_envs"])
    fb, pb = (4, 4) if args.obs_format == "f32" else (1, 2)
    per_env = cfg.grid * cfg.grid * (2 * fb + (0 if args.no_potential else pb)) + 4096
    budget = int(0.7 * torch.cuda.get_device_properties(dev).total_memory)
    if not args.envs and strong and n * per_env > budget:
        n = pr["n_envs"] // pr["gpus"]
        strong = False
    return cfg, n, strong


def _free_port() -> int:
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(n: int, cmd=None) -> int:
    """`bench.py --gpus N` without torchrun: start N rank children of this same command line, one
    per GPU, with the torchrun environment variables set, and wait for all of them.  Called before
    torch is imported, so this parent never initialises the GPU (no HIP call, no exec)."""
    import signal
    import subprocess
    port = _free_port()
    cmd = cmd or [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FFMP_BENCH_LAUNCHER="1")
        procs.append(subprocess.Popen(cmd, env=env))
    rc = 0
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                code = p.poll()
                if code is None:
                    continue
                pending.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
                    for q in pending:  # one rank failed: the others would wait in a collective forever
                        q.send_signal(signal.SIGTERM)
            time.sleep(0.2)
    except KeyboardInterrupt:
        for p in procs:
            p.send_signal(signal.SIGTERM)
        rc = 130
    for p in procs:
        try:
            p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            p.kill()
    return rc


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    import torch
    import torch.distributed as dist
    from flow_field_based_motion_planner_amd.vec_env import FFMPVec

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"error: WORLD_SIZE={world} but --gpus={args.gpus} (run with torchrun --nproc-per-node {args.gpus}, "
              f"or without WORLD_SIZE set and bench.py starts the ranks)", file=sys.stderr)
        sys.exit(2)
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", local % max(ndev, 1))
    torch.cuda.set_device(dev)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    pg_world = dist.get_world_size() if world > 1 else 1  # as the collective backend sees it
    if pg_world != args.gpus:
        print(f"error: the process group has {pg_world} ranks, --gpus={args.gpus}", file=sys.stderr)
        sys.exit(2)

    name = args.config
    cfg, n, strong = _leg_size(name, args, world, dev)
    K, W = args.steps, args.warmup
    off0 = rank * n if args.env_offset is None else args.env_offset + rank * n
    leg, env = run_leg(args, name, cfg, n, off0, K, W, dev, world, rank, strong, True)
    traffic, traffic_source = load_traffic(name, leg["per_launch_envs"], env.frame_window, env.ring, env.fused,
                                           args.obs_format, (leg["graph"] or {}).get("steps_per_replay", 0),
                                           bool((leg["graph"] or {}).get("skewed", False)))
    _release(env)
    env = None

    # the compact layout (N = 1), before the strong leg: that one's ring takes most of the HBM, and
    # the pieces of rings this process dropped stay mapped
    compact = None
    if world == 1 and args.obs_format == "f32" and args.compact_steps > 0 and not args.tuning \
            and not args.no_potential and not args.flow:
        torch.cuda.empty_cache()
        compact = time_compact_child(name, args.compact_steps, args.seed)
        if compact is None:  # in this process instead (after the float32 instance: placement-dependent)
            compact = time_compact(FFMPVec, name, cfg, n, dev, args.compact_steps, 10, args.seed)
            compact["process"] = "this process, after the float32 instance"

    # second leg: the strong-scaling preset split over the ranks (C4's 65,536 envs over
    # 1, 2, 4, 8 GPUs), so one driver command yields both curves
    strong_leg = None
    if args.strong_config != "none" and args.strong_config != name and not args.tuning:
        scfg, sn, s_strong = _leg_size(args.strong_config, args, world, dev)
        if s_strong:
            from flow_field_based_motion_planner_amd.distributed import shard_range
            from flow_field_based_motion_planner_amd.config import PRESETS
            off, sn = shard_range(PRESETS[args.strong_config]["n_envs"], world, rank)
            strong_leg, env = run_leg(args, args.strong_config, scfg, sn, off, args.strong_steps or K, W, dev,
                                      world, rank, True, False)
            _release(env)
            env = None
            strong_leg.pop("raster_autotune", None)
            strong_leg.pop("per_launch_envs", None)

    if rank == 0:
        # traffic: the PMC-measured HBM bytes per launch of this launch kind, looked up from the
        # committed rocprofv3 summary named by traffic_source (bench.py runs no counters itself)
        rl = dict(leg["roofline"], traffic=traffic, traffic_source=traffic_source)
        out = {
            "metric": METRIC,
            "value": leg["value"],
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": leg["ms_per_step"],
            "higher_is_better": True,
            "scaling": leg["scaling"],
            "vs_baseline": None,
            "dtype": "f32" if args.obs_format == "f32" else "u8 frames / f16 potential (f32 compute)",
            "data": "synthetic",
            "config": {"workload": name, "n_envs_total": leg["n_envs_total"], "n_envs_per_gpu": n, "env_offset": off0,
                       "grid": cfg.grid,
                       "n_obst": cfg.n_obst, "moving": bool(cfg.moving), "n_beams": cfg.n_beams,
                       "potential": not args.no_potential, "flow": bool(args.flow), "obs_format": args.obs_format,
                       "frame_window": leg["frame_window"], "ring": leg["ring"], "fused": leg["fused"],
                       "graph": leg["graph"],
                       "parallelism": f"env-shard x{world}",
                       "comm": (args.dist_backend if world > 1 else "none"), "world_size_backend": pg_world,
                       "launcher": ("bench.py" if os.environ.get("FFMP_BENCH_LAUNCHER") else
                                    "torchrun" if "WORLD_SIZE" in os.environ else "none")},
            "roofline": rl,
            "per_rank_ms_per_step": leg["per_rank_ms_per_step"],
            "construct_s": leg["construct_s"],
            "per_rank_construct_s": leg["per_rank_construct_s"],
            # every rank's kernel time, roofline fraction, launch choice and ring pairing (RANK_FIELDS)
            "per_rank": leg["per_rank"],
            "hbm_bytes": leg["hbm_bytes"],
            "hbm_in_use_bytes": leg["hbm_in_use_bytes"],
            # HBM the process holds beyond the instance (torch context, caches); round 3 parked ~65 GB
            # of unchosen ring pieces here, now released after construction (pool_released_bytes)
            "hbm_beyond_instance_bytes": leg["hbm_in_use_bytes"] - leg["hbm_bytes"],
            "pool_released_bytes": leg["pool_released_bytes"],
            "raster_ms_per_step": leg["raster_ms_per_step"],
            "step_ms_events": leg["step_ms_events"],
            "pipeline_slices": leg["pipeline_slices"],
            "raster_autotune": leg["raster_autotune"],
            "hbm_roofline_pct_whole_step": leg["hbm_roofline_pct_whole_step"],
        }
        if leg.get("closed_loop") is not None:
            out["closed_loop"] = leg["closed_loop"]
        if strong_leg is not None:
            out["strong"] = strong_leg
        if compact is not None:
            out["compact_layout"] = compact
        if world == 1 and args.cpu_seconds > 0:
            out["cpu_baseline"] = cpu_baseline(cfg, args.cpu_seconds, args.cpu_threads)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
