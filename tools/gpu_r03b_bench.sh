#!/bin/bash
# round 3 (second session): the default bench as the driver runs it (compact leg in a child process)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r03b_bench_child.log 2>&1 || { tail -20 gpurun_out/r03b_bench_child.log; exit 1; }
tail -1 gpurun_out/r03b_bench_child.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['compact_layout']; r=d['roofline']; s=d.get('strong') or {}
print('f32', round(d['value']/1e6,3), r['kernel'], round(r['kernel_ms'],4), round(r['frac'],3), '| strong', round(s.get('value',0)/1e6,3), '| compact', round(c['value']/1e6,2), c['kernel'], round(c['kernel_ms'],4), round(c['frac'],3), c['shape'], c['fused'], c.get('process'))"
