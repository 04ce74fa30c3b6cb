#!/bin/bash
# SQ counters of the learner's MFMA convolutions at B = 256 (tools/conv_probe.py): MFMA busy cycles against
# the cycles the chip actually ran (GRBM_GUI_ACTIVE / 8 per XCD), wave states, LDS bank conflicts.
# usage: gpu_conv_pmc.sh <out-dir name>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE \
  --kernel-include-regex 'conv_' --kernel-trace --output-format csv -d $O/run -o run -- \
  python3 $R/tools/conv_probe.py 256 --mfma-only > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
cd $R && python3 - "$1" <<'PY'
import csv, glob, collections, sys
f = sorted(glob.glob(f"gpurun_out/{sys.argv[1]}/run/**/run_counter_collection.csv", recursive=True))[-1]
by = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    by[(int(r["Dispatch_Id"]), r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
kinds = collections.defaultdict(list)
for (d, name), c in sorted(by.items()):
    kinds[name].append(c)
print("kernel | dispatches | MFMA busy / (GRBM/8 cycles x 4 SIMD x 256 CU) | GRBM/8 cycles | parked / issue-stall / issuing (of wave cycles) | LDS bank-conflict / LDS-active cycles")
for name, lst in kinds.items():
    a = collections.Counter()
    for c in lst[1:] or lst:
        a.update(c)
    n = max(len(lst) - 1, 1)
    a = {k: v / n for k, v in a.items()}
    cyc = a.get("GRBM_GUI_ACTIVE", 0) / 8
    mfma = a.get("SQ_VALU_MFMA_BUSY_CYCLES", 0)
    wc = a.get("SQ_WAVE_CYCLES", 1)
    util = mfma / (cyc * 4 * 256) if cyc else 0
    print(f"{name[:70]} | {len(lst)} | {util:.3f} | {cyc:.4g} | {a.get('SQ_WAIT_ANY',0)/wc:.2f} / {a.get('SQ_WAIT_INST_ANY',0)/wc:.2f} / {a.get('SQ_ACTIVE_INST_ANY',0)/wc:.2f} | {a.get('SQ_LDS_BANK_CONFLICT',0)/max(a.get('SQ_LDS_IDX_ACTIVE',1),1):.3f}")
PY
grep mfma $O/probe.log
