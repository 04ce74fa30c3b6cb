#!/bin/bash
# round 3 (second session): the driver's bench command line on the final code, two fresh processes
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r03b_final_bench_$i.log 2>&1 || { tail -20 gpurun_out/r03b_final_bench_$i.log; exit 1; }
  tail -1 gpurun_out/r03b_final_bench_$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['compact_layout']; r=d['roofline']; s=d.get('strong') or {}; b=d['cpu_baseline']
print('f32', round(d['value']/1e6,3), r['kernel'], round(r['kernel_ms'],4), round(r['frac'],3), d['raster_autotune']['shape_newest'], '| strong', round(s.get('value',0)/1e6,3), '| compact', round(c['value']/1e6,2), round(c['kernel_ms'],4), round(c['frac'],3), c['shape'], '| cpu', round(b['value']/1e3,1), 'K')"
done
