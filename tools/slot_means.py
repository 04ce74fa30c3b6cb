"""Per-slot mean of the timed raster launches of bench.py --dump-launches runs (C3, seamless W = 8):
the bench resets, runs --warmup steps, then times --steps; step j after the reset writes physical
slot (j + 2) % W (FFMPVec._slot_written).  usage: python tools/slot_means.py <warmup> <run.err> ..."""
import re
import sys

warm, W = int(sys.argv[1]), 8
for path in sys.argv[2:]:
    line = next((ln for ln in open(path) if ln.startswith("raster ms per launch:")), None)
    if line is None:
        print(path, "no dump")
        continue
    ms = [float(v) for v in line.split(":", 1)[1].split()]
    per = {}
    for j, v in enumerate(ms):
        per.setdefault((warm + j + 2) % W, []).append(v)
    means = [sum(per[s]) / len(per[s]) for s in sorted(per)]
    print(f"{path.split('/')[-1]:22s} mean {sum(ms) / len(ms):.4f}  slots " + " ".join(f"{m:.3f}" for m in means)
          + f"  spread {max(means) / min(means):.3f}")
