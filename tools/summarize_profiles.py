#!/usr/bin/env python3
"""Turn the rocprofv3 CSVs written by tools/gpu_profile.sh into committed evidence.

  profiles/<tag>_<cfg>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (bench.py, 50 steps)
  profiles/<tag>_<cfg>_bench.json         the bench.py JSON line printed under that trace
  profiles/<tag>_<cfg>_pmc.json           per-kernel WRITE_SIZE / FETCH_SIZE (separate --pmc passes),
                                          converted to bytes per launch with the gfx950 correction
                                          (FETCH_SIZE counts half of wide streaming reads: x2);
                                          raster: mean over the pass's timed launches (the frame
                                          window mixes full and newest-only launches), other
                                          kernels: median over dispatches
  profiles/pmc_traffic_<cfg>[_fused][_graph].json what bench.py reads for roofline.traffic (_graph:
                                          per replay of the timed HIP graph, its env kernels + rasters)
"""
import csv
import glob
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "gpurun_out", "prof")
OUT = os.path.join(ROOT, "profiles")


def find(pattern):
    hits = sorted(glob.glob(os.path.join(PROF, "**", pattern), recursive=True))
    return hits[-1] if hits else None


def bench_json(log):
    for line in open(log):
        if line.startswith("{"):
            return json.loads(line)
    return None


def counters(path, name):
    """kernel -> counter values in dispatch order."""
    per = {}
    with open(path) as f:
        rows = sorted((r for r in csv.DictReader(f) if r.get("Counter_Name") == name),
                      key=lambda r: int(r["Dispatch_Id"]))
    for row in rows:
        k = row["Kernel_Name"]
        # "raster_kernel" = the timed kernel: raster_kernel or step_raster_kernel (fused step);
        # "skew_kernel": the skewed step's launch (raster of step i + env step of step i + 1)
        key = ("skew_kernel" if "skew_kernel" in k else "raster_kernel" if "raster_kernel" in k else
               "env_kernel" if "env_kernel" in k else k)
        per.setdefault(key, []).append(float(row["Counter_Value"]))
    return per


def graph_steps(bj) -> int:
    """Steps per replay when bench.py timed HIP-graph replays (config.graph), else 0."""
    return int(((bj or {}).get("config", {}).get("graph") or {}).get("steps_per_replay", 0) or 0)


def timed_launches(log):
    """Raster (or one-launch step) dispatches bench.py timed: one per step (per slice), or with
    graph replays one per replayed step."""
    bj = bench_json(log) if os.path.exists(log) else None
    if not bj:
        return None
    g = graph_steps(bj)
    if g:
        return bj["config"]["graph"]["replays"] * g + bj["config"]["graph"].get("remainder_steps", 0)
    return bj["steps"] * bj["roofline"].get("launches_per_step", 1)


def step_kernels(path, name):
    """(kernel key, value) of the step's own dispatches (env / raster / skew kernels) in dispatch order."""
    with open(path) as f:
        rows = sorted((r for r in csv.DictReader(f) if r.get("Counter_Name") == name and
                       any(t in r["Kernel_Name"] for t in ("env_kernel", "raster_kernel", "skew_kernel"))),
                      key=lambda r: int(r["Dispatch_Id"]))
    return [("skew_kernel" if "skew_kernel" in r["Kernel_Name"] else "raster_kernel" if "raster_kernel" in
             r["Kernel_Name"] else "env_kernel", float(r["Counter_Value"])) for r in rows]


def replay_dispatches(bj, gs):
    """(dispatches per full replay, dispatches of the remainder replay) of bench.py's timed graphs: per
    step an env kernel + a raster (two-launch), one step kernel (fused), or env(0) + (gs - 1) skewed
    launches + raster(gs - 1) (skewed)."""
    g = bj["config"]["graph"]
    rem = g.get("remainder_steps", 0)
    if bj["config"].get("fused"):
        return gs, rem
    if g.get("skewed"):
        return gs + 1, (rem + 1 if rem and rem % 2 == 0 else 2 * rem)
    return 2 * gs, 2 * rem


def per_launch(vals, key, k, graph=False):
    if (key == "raster_kernel" or (graph and key == "env_kernel")) and k:
        tail = vals[-k:]
        return sum(tail) / len(tail)
    return statistics.median(vals)


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    cfg = sys.argv[2] if len(sys.argv) > 2 else "C3"  # label: <workload>[_u8f16]
    os.makedirs(OUT, exist_ok=True)
    stats = find(f"trace_{cfg}/**/run_kernel_stats.csv") or find("run_kernel_stats.csv")
    if stats:
        shutil.copy(stats, os.path.join(OUT, f"{tag}_{cfg}_kernel_stats.csv"))
    bj = bench_json(os.path.join(PROF, f"bench_trace_{cfg}.log"))
    if bj:
        with open(os.path.join(OUT, f"{tag}_{cfg}_bench.json"), "w") as f:
            json.dump(bj, f, indent=1)
    w = counters(find(f"pmcw_{cfg}/**/run_counter_collection.csv"), "WRITE_SIZE")
    r = counters(find(f"pmcf_{cfg}/**/run_counter_collection.csv"), "FETCH_SIZE")
    kw = timed_launches(os.path.join(PROF, f"bench_pmcw_{cfg}.log"))
    kf = timed_launches(os.path.join(PROF, f"bench_pmcf_{cfg}.log"))
    gs = graph_steps(bj)
    pm = {"workload": cfg, "units": "bytes per launch (raster: mean over the timed launches; others: median)",
          "correction": "WRITE_SIZE*1024 exact for 16-B/lane streaming stores; FETCH_SIZE*1024*2 (gfx950 halves wide "
                        "streaming reads, MI355X_MICROARCH.md HBM section)", "kernels": {}}
    for k in sorted(set(w) | set(r)):
        wb = per_launch(w.get(k, [0.0]), k, kw, bool(gs)) * 1024
        fb = per_launch(r.get(k, [0.0]), k, kf, bool(gs)) * 1024 * 2
        pm["kernels"][k] = {"write_bytes": wb, "fetch_bytes_corrected": fb, "hbm_bytes": wb + fb,
                            "dispatches": len(w.get(k, []))}
    if bj:
        n = bj["config"]["n_envs_per_gpu"]
        alg = bj["roofline"]["algorithmic_bytes_per_launch"]
        pm["n_envs"] = n
        pm["frame_window"] = bj["config"].get("frame_window", 2)
        pm["ring"] = bj["config"].get("ring", "wrap" if pm["frame_window"] > 2 else "contiguous")
        pm["fused"] = bool(bj["config"].get("fused", False))
        pm["obs_format"] = bj["config"].get("obs_format", "f32")
        pm["timed_kernel"] = bj["roofline"].get("kernel", "raster_kernel")
        pm["raster_algorithmic_bytes_per_launch"] = alg
        if "raster_kernel" in pm["kernels"]:
            hb = pm["kernels"]["raster_kernel"]["hbm_bytes"]
            sfx = "_fused" if pm["fused"] else ""
            rec = {"n_envs": n, "frame_window": pm["frame_window"], "ring": pm["ring"], "fused": pm["fused"],
                   "obs_format": bj["config"].get("obs_format", "f32"), "raster_hbm_bytes_per_launch": hb,
                   "source": f"{tag}_{cfg}_pmc.json"}
            if gs and bj["config"]["graph"].get("skewed"):  # (a skew trial alone leaves skew_kernel rows too)
                # a skewed graph: the HBM bytes of the timed replays' own dispatches, per replay
                per_rep, rem_d = replay_dispatches(bj, gs)
                R = bj["config"]["graph"]["replays"]
                tot = []
                for name, path, scale in (("WRITE_SIZE", find(f"pmcw_{cfg}/**/run_counter_collection.csv"), 1024),
                                          ("FETCH_SIZE", find(f"pmcf_{cfg}/**/run_counter_collection.csv"), 2048)):
                    rows = step_kernels(path, name)
                    timed = rows[len(rows) - rem_d - R * per_rep:len(rows) - rem_d]
                    tot.append(sum(v for _, v in timed) * scale / R)
                pm["graph_steps"] = gs
                pm["skewed"] = True
                pm["step_graph_hbm_bytes_per_replay"] = sum(tot)
                pm["step_graph_traffic_over_algorithmic"] = sum(tot) / alg
                rec.update(graph_steps=gs, step_graph_hbm_bytes_per_replay=sum(tot), skewed=True)
                sfx += "_graph"
            elif gs:
                # the timed unit is one replay of gs whole steps: their env kernels and rasters
                eb = pm["kernels"].get("env_kernel", {}).get("hbm_bytes", 0.0)
                pm["graph_steps"] = gs
                pm["step_graph_hbm_bytes_per_replay"] = gs * (hb + eb)
                pm["step_graph_traffic_over_algorithmic"] = gs * (hb + eb) / alg
                rec.update(graph_steps=gs, step_graph_hbm_bytes_per_replay=gs * (hb + eb))
                sfx += "_graph"
            else:
                pm["raster_traffic_over_algorithmic"] = hb / alg
            # bench.py looks the one-launch step up under its own label first
            with open(os.path.join(OUT, f"pmc_traffic_{cfg}{sfx}.json"), "w") as f:
                json.dump(rec, f, indent=1)
    trace = find(f"trace_{cfg}/**/run_kernel_trace.csv")
    if trace and bj and gs:
        # each timed replay = gs consecutive steps of (env kernel, raster) or (one-launch step):
        # its duration in the trace = first dispatch's start to last dispatch's end
        rows = [r for r in csv.DictReader(open(trace)) if "raster_kernel" in r["Kernel_Name"] or
                "env_kernel" in r["Kernel_Name"] or "skew_kernel" in r["Kernel_Name"]]
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        per_rep, rem = replay_dispatches(bj, gs)  # a shorter last replay: rem dispatches
        R = bj["config"]["graph"]["replays"]
        timed = rows[len(rows) - rem - R * per_rep:len(rows) - rem]
        reps = [timed[i * per_rep:(i + 1) * per_rep] for i in range(R)]
        gaps = [int(b_["Start_Timestamp"]) - int(a_["End_Timestamp"]) for rp in reps for a_, b_ in zip(rp, rp[1:])]
        pm["graph_inter_kernel_gap_avg_ns"] = sum(gaps) / max(len(gaps), 1)
        durs = [int(rp[-1]["End_Timestamp"]) - int(rp[0]["Start_Timestamp"]) for rp in reps]
        busy = [sum(int(x["End_Timestamp"]) - int(x["Start_Timestamp"]) for x in rp) for rp in reps]
        pm["graph_timed_replays"] = R
        pm["graph_replay_avg_ns_kernel_trace"] = sum(durs) / len(durs)
        pm["graph_replay_kernel_busy_avg_ns"] = sum(busy) / len(busy)  # the kernels' own durations
        pm["graph_replay_avg_ns_bench_events"] = bj["roofline"]["kernel_ms"] * 1e6
        pm["trace_vs_events"] = pm["graph_replay_avg_ns_kernel_trace"] / pm["graph_replay_avg_ns_bench_events"]
        ras = [int(x["End_Timestamp"]) - int(x["Start_Timestamp"]) for x in timed if "raster_kernel" in x["Kernel_Name"]]
        env_ = [int(x["End_Timestamp"]) - int(x["Start_Timestamp"]) for x in timed if "env_kernel" in x["Kernel_Name"]]
        skw = [int(x["End_Timestamp"]) - int(x["Start_Timestamp"]) for x in timed if "skew_kernel" in x["Kernel_Name"]]
        pm["raster_avg_ns_kernel_trace"] = sum(ras) / max(len(ras), 1)
        if env_:
            pm["env_kernel_avg_ns_kernel_trace"] = sum(env_) / len(env_)
        if skw:
            pm["skew_kernel_avg_ns_kernel_trace"] = sum(skw) / len(skw)
        pm["raster_kernel_name"] = timed[-1]["Kernel_Name"]
    elif trace and bj:
        # the last (steps x launches_per_step) raster dispatches are exactly the launches bench.py
        # timed; earlier ones are warm-up and the per-instance launch-shape autotune
        rows = [r for r in csv.DictReader(open(trace)) if "raster_kernel" in r["Kernel_Name"]]
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        k = bj["steps"] * bj["roofline"].get("launches_per_step", 1)
        timed = rows[-k:]
        durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in timed]
        pm["raster_timed_dispatches"] = len(durs)
        pm["raster_kernel_name"] = timed[-1]["Kernel_Name"]
        pm["raster_avg_ns_kernel_trace"] = sum(durs) / len(durs)
        pm["raster_avg_ns_bench_events"] = bj["roofline"]["kernel_ms"] * 1e6
        pm["trace_vs_events"] = pm["raster_avg_ns_kernel_trace"] / pm["raster_avg_ns_bench_events"]
    with open(os.path.join(OUT, f"{tag}_{cfg}_pmc.json"), "w") as f:
        json.dump(pm, f, indent=1)
    print(json.dumps(pm, indent=1))


if __name__ == "__main__":
    main()
