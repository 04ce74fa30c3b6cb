#!/bin/bash
# Raster tuning sweep on the GPU box: write-BW probe, parity, bench per (cells/block, store flavour).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
hipcc --offload-arch=gfx950 -O3 -o /tmp/hbm_write_probe tools/hbm_write_probe.hip > /dev/null 2>&1 || exit 1
echo "== probe"; timeout -k 10 300 /tmp/hbm_write_probe 256 32768 > gpurun_out/probe.log 2>&1 || exit 1
cat gpurun_out/probe.log
echo "== parity"; timeout -k 10 600 python tests/parity_report.py > gpurun_out/parity.log 2>&1 || exit 1
grep -E '^\[' gpurun_out/parity.log
: > gpurun_out/tune.log
for cfg in C3 C2; do
for cpb in 4096 8192 16384 32768; do
for nt in 1 0; do
  echo "== $cfg cpb=$cpb nt=$nt" >> gpurun_out/tune.log
  FFMP_RASTER_CPB=$cpb FFMP_RASTER_NT=$nt timeout -k 10 300 python bench.py --config $cfg --steps 40 --warmup 5 --cpu-seconds 0 >> gpurun_out/tune.log 2>&1 || exit 1
done; done; done
python - <<'PY'
import json
cur = None
for line in open("gpurun_out/tune.log"):
    if line.startswith("=="):
        cur = line.strip()
    elif line.startswith("{"):
        d = json.loads(line)
        print(cur, "value %.3e" % d["value"], "raster_ms %.3f" % d["roofline"]["kernel_ms"], "GB/s %.0f" % d["roofline"]["achieved"], "env_ms %.3f" % d["env_kernel_ms"])
PY
