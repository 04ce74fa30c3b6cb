#!/bin/bash
# SQ counters of env_kernel (ffmp_step_state) at C3: issue-bound (VALU) or waiting (memory/LDS)?
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/epmc
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE \
  --kernel-include-regex 'env_kernel' --output-format csv -d $R/gpurun_out/epmc/run -o run -- \
  python3 $R/tools/env_kernel_breakdown.py --preset C3 base > $R/gpurun_out/epmc/log.txt 2>&1 || exit 1
cd $R && python3 - <<'PY'
import csv, glob, collections
f = sorted(glob.glob("gpurun_out/epmc/run/**/run_counter_collection.csv", recursive=True))[-1]
by = collections.defaultdict(dict)
for r in csv.DictReader(open(f)):
    by[(int(r["Dispatch_Id"]), r["Kernel_Name"][:60])][r["Counter_Name"]] = float(r["Counter_Value"])
last = sorted(by.items())[-20:]
agg = collections.Counter()
for _, c in last:
    agg.update(c)
a = {k: v / len(last) for k, v in agg.items()}
print(last[-1][0][1])
for k in sorted(a):
    print(f"   {k:22s} {a[k]:.4g}")
wc = a.get("SQ_WAVE_CYCLES", 1)
print(f"   parked {a.get('SQ_WAIT_ANY',0)/wc:.3f}  issue-stall {a.get('SQ_WAIT_INST_ANY',0)/wc:.3f}  issuing {a.get('SQ_ACTIVE_INST_ANY',0)/wc:.3f}  "
      f"VALU/wave {a.get('SQ_INSTS_VALU',0)/max(a.get('SQ_WAVES',1),1):.0f}  SALU/wave {a.get('SQ_INSTS_SALU',0)/max(a.get('SQ_WAVES',1),1):.0f}")
cyc = a.get("GRBM_GUI_ACTIVE", 0) / 8
print(f"   cycles/launch ~{cyc:.3g}; VALU capacity 256x4xcycles/4 = {256*4*cyc/4:.3g} vs {a.get('SQ_INSTS_VALU',0):.3g} issued")
PY
