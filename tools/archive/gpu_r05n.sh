#!/bin/bash
# Round 5: does a pipelined step graph overlap its env kernels with the rasters?  Kernel trace of bench.py
# C2 (graph replays, pipelined), then the overlap of env_kernel and raster_kernel intervals.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05n
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 $R/bench.py --config C2 --steps 32 --warmup 8 --cpu-seconds 0 --strong-config none --compact-steps 0 --fused off > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
cd $R && python3 - <<'PY'
import csv, glob
f = sorted(glob.glob("gpurun_out/r05n/trace/**/run_kernel_trace.csv", recursive=True))[-1]
rows = list(csv.DictReader(open(f)))
ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:40]) for r in rows
      if "env_kernel" in r["Kernel_Name"] or "raster_kernel" in r["Kernel_Name"]]
ks.sort()
last = ks[-80:]
ov = 0
for i in range(1, len(last)):
    if last[i][0] < last[i - 1][1]:
        ov += 1
print("last 80 env/raster kernels: overlapping starts", ov)
t0 = last[0][0]
for s, e, n in last[-24:]:
    print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f} us  {n}")
PY
