#!/bin/bash
# VALU busy % of the kernels under bench.py (C3, C5 share): is the raster store-bound or VALU-bound?
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/valu
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import sys; sys.path.insert(0,'$R'); import __graft_entry__ as g; g.build()" || exit 1
for CFG in C3 C5; do
  timeout -k 10 600 rocprofv3 --pmc VALUBusy SALUBusy --kernel-include-regex 'raster_kernel|env_kernel' --output-format csv \
    -d $R/gpurun_out/valu/$CFG -o run -- python3 $R/bench.py --config $CFG --steps 14 --warmup 2 --cpu-seconds 0 \
    > $R/gpurun_out/valu/bench_$CFG.log 2>&1 || exit 1
done
cd $R && python3 - <<'PY'
import csv, glob, statistics
for cfg in ("C3", "C5"):
    f = sorted(glob.glob(f"gpurun_out/valu/{cfg}/**/run_counter_collection.csv", recursive=True))[-1]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Dispatch_Id"]))
    for k in ("raster_kernel", "env_kernel"):
        for c in ("VALUBusy", "SALUBusy"):
            v = [float(r["Counter_Value"]) for r in rows if k in r["Kernel_Name"] and r["Counter_Name"] == c][-14:]
            if v:
                print(f"{cfg} {k:13s} {c}: mean {statistics.mean(v):6.2f} %  (last {len(v)} dispatches)")
PY
