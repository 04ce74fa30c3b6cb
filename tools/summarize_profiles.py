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
  profiles/pmc_traffic_<cfg>[_fused].json what bench.py reads for roofline.traffic
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
        # "raster_kernel" = the timed kernel: raster_kernel or step_raster_kernel (fused step)
        key = "raster_kernel" if "raster_kernel" in k else ("env_kernel" if "env_kernel" in k else k)
        per.setdefault(key, []).append(float(row["Counter_Value"]))
    return per


def timed_launches(log):
    bj = bench_json(log) if os.path.exists(log) else None
    return bj["steps"] * bj["roofline"].get("launches_per_step", 1) if bj else None


def per_launch(vals, key, k):
    if key == "raster_kernel" and k:
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
    pm = {"workload": cfg, "units": "bytes per launch (raster: mean over the timed launches; others: median)",
          "correction": "WRITE_SIZE*1024 exact for 16-B/lane streaming stores; FETCH_SIZE*1024*2 (gfx950 halves wide "
                        "streaming reads, MI355X_MICROARCH.md HBM section)", "kernels": {}}
    for k in sorted(set(w) | set(r)):
        wb = per_launch(w.get(k, [0.0]), k, kw) * 1024
        fb = per_launch(r.get(k, [0.0]), k, kf) * 1024 * 2
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
            pm["raster_traffic_over_algorithmic"] = hb / alg
            # bench.py looks the one-launch step up under its own label first
            sfx = "_fused" if pm["fused"] else ""
            with open(os.path.join(OUT, f"pmc_traffic_{cfg}{sfx}.json"), "w") as f:
                json.dump({"n_envs": n, "frame_window": pm["frame_window"], "ring": pm["ring"], "fused": pm["fused"],
                           "obs_format": bj["config"].get("obs_format", "f32"),
                           "raster_hbm_bytes_per_launch": hb,
                           "source": f"{tag}_{cfg}_pmc.json"}, f, indent=1)
    trace = find(f"trace_{cfg}/**/run_kernel_trace.csv")
    if trace and bj:
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
