"""Per-process summary of rocprofv3 counter CSVs under gpurun_out/tlb/<run>/: raster GB/s from
dispatch timestamps + mean counter values (last 6 raster dispatches)."""
import csv
import glob
import os
import statistics
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/tlb"
BYTES = 25788678144  # C3 raster algorithmic bytes per launch
for d in sorted(glob.glob(os.path.join(root, "*"))):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        continue
    per = {}
    times = {}
    for f in files:
        for row in csv.DictReader(open(f)):
            if "raster_kernel" not in row["Kernel_Name"]:
                continue
            did = int(row["Dispatch_Id"])
            per.setdefault(row["Counter_Name"], {})[did] = float(row["Counter_Value"])
            times[did] = (int(row["Start_Timestamp"]), int(row["End_Timestamp"]))
    ids = sorted(times)[-6:]
    gbs = statistics.median(BYTES / (times[i][1] - times[i][0]) for i in ids)
    vals = {k: statistics.median(v[i] for i in ids if i in v) for k, v in per.items()}
    print(os.path.basename(d), f"raster {gbs:.0f} GB/s", " ".join(f"{k}={v:.3g}" for k, v in sorted(vals.items())))
