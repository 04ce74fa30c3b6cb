#!/bin/bash
# round 4: where the learner loop's time goes now (examples/train_vec.py --amp, 60 loop steps = 60
# updates after 3 warm-up), rocprofv3 kernel trace + stats; per-update kernel split
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04p
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python3 $R/examples/train_vec.py --amp --steps 60 > $O/train.log 2>&1 || { tail -20 $O/train.log; exit 1; }
tail -1 $O/train.log
cd $R && python3 - <<'PY'
import csv, glob
f = sorted(glob.glob("gpurun_out/r04p/trace/**/run_kernel_stats.csv", recursive=True))[-1]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
U = 63
print(f"total kernel time {tot/1e6:.1f} ms, {tot/1e6/U:.2f} ms per loop step ({U} incl. warm-up)")
print(" share  ms/step  calls/step  mean_us  kernel")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:40]:
    t = float(r["TotalDurationNs"])
    print(f"{100*t/tot:5.1f} {t/1e6/U:8.3f} {int(r['Calls'])/U:10.1f} {float(r['AverageNs'])/1e3:8.1f}  {r['Name'][:110]}")
PY
