#!/usr/bin/env python3
"""Per-kernel summary (calls, total / mean ms, share) of a rocprofv3 rocpd database, optionally only
the dispatches after the first `--skip-s` seconds of GPU activity (warm-up / MIOpen search)."""
import argparse
import sqlite3
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--skip-s", type=float, default=0.0)
ap.add_argument("--top", type=int, default=25)
a = ap.parse_args()
db = sqlite3.connect(a.db)
rows = db.execute("select k.kernel_name, d.start, d.end from rocpd_kernel_dispatch d "
                  "join rocpd_info_kernel_symbol k on d.kernel_id = k.id").fetchall()
t0 = min(r[1] for r in rows)
per = defaultdict(lambda: [0, 0.0])
for name, s, e in rows:
    if (s - t0) * 1e-9 < a.skip_s:
        continue
    per[name][0] += 1
    per[name][1] += (e - s) * 1e-6
tot = sum(v[1] for v in per.values())
print(f"{'share':>6} {'total ms':>10} {'calls':>6} {'mean ms':>9}  kernel")
for name, (n, ms) in sorted(per.items(), key=lambda kv: -kv[1][1])[:a.top]:
    print(f"{100 * ms / tot:6.1f} {ms:10.2f} {n:6d} {ms / n:9.4f}  {name[:110]}")
print(f"total kernel time {tot:.1f} ms over {sum(v[0] for v in per.values())} dispatches")
