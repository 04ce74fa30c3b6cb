#!/bin/bash
# write-BW probe and bench.py in the SAME call (same box) for A/B comparisons
set -o pipefail
mkdir -p gpurun_out
hipcc --offload-arch=gfx950 -O3 -o /tmp/hbm_write_probe tools/hbm_write_probe.hip > /dev/null 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > /dev/null 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 300 /tmp/hbm_write_probe 256 32768 > gpurun_out/probe_$r.log 2>&1 || exit 1
  grep -E 'three_planes.*cpb=4096|Memset|P=3 V=1 BS=256' gpurun_out/probe_$r.log
  timeout -k 10 300 python bench.py --steps 100 --warmup 10 --cpu-seconds 0 > gpurun_out/bench_ab_$r.log 2>&1 || exit 1
  python -c "import json;d=json.loads([l for l in open('gpurun_out/bench_ab_$r.log') if l.startswith('{')][0]);print('bench', '%.3e'%d['value'], d['roofline']['kernel_ms'], '%.0f'%d['roofline']['achieved'])"
done
rocm-smi --showmeminfo vram 2>/dev/null | head -5; rocm-smi --showclocks 2>/dev/null | grep -iE 'mclk|fclk' | head
