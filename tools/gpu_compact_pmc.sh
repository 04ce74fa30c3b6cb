#!/bin/bash
# Why is the compact raster (obs_format=u8f16) at ~0.5 of HBM peak?  One SQ counter pass over
# bench.py C3 --obs-format u8f16 (and f32 for comparison): wave cycles split into
# parked (WAIT_ANY: s_waitcnt / barrier), issue-stalled (WAIT_INST_ANY) and issuing (ACTIVE_INST_ANY),
# plus VALU instructions per wave.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/cpmc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import sys; sys.path.insert(0,'$R'); import __graft_entry__ as g; g.build()" || exit 1
for FMT in u8f16 f32; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE \
    --kernel-include-regex 'raster_kernel' --output-format csv -d $R/gpurun_out/cpmc/$FMT -o run -- \
    python3 $R/bench.py --config C3 --obs-format $FMT --fused off --steps 8 --warmup 2 --cpu-seconds 0 \
    > $R/gpurun_out/cpmc/bench_$FMT.log 2>&1 || exit 1
done
cd $R && python3 - <<'PY'
import csv, glob, collections
for fmt in ("u8f16", "f32"):
    f = sorted(glob.glob(f"gpurun_out/cpmc/{fmt}/**/run_counter_collection.csv", recursive=True))[-1]
    by = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        by[(int(r["Dispatch_Id"]), r["Kernel_Name"][:60])][r["Counter_Name"]] = float(r["Counter_Value"])
    last = sorted(by.items())[-8:]
    agg = collections.Counter()
    for _, c in last:
        agg.update(c)
    n = len(last)
    a = {k: v / n for k, v in agg.items()}
    print(fmt, last[-1][0][1])
    for k in sorted(a):
        print(f"   {k:22s} {a[k]:.4g}")
    wc = a.get("SQ_WAVE_CYCLES", 1)
    print(f"   parked {a.get('SQ_WAIT_ANY',0)/wc:.3f}  issue-stall {a.get('SQ_WAIT_INST_ANY',0)/wc:.3f}  issuing {a.get('SQ_ACTIVE_INST_ANY',0)/wc:.3f}  "
          f"VALU/wave {a.get('SQ_INSTS_VALU',0)/max(a.get('SQ_WAVES',1),1):.0f}  SALU/wave {a.get('SQ_INSTS_SALU',0)/max(a.get('SQ_WAVES',1),1):.0f}")
PY
