#!/bin/bash
# round 3 (second session): per-launch raster times of the driver's command line (20 timed steps after
# 5 warm-up steps), three fresh processes, to see where a slow run's time goes
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --dump-launches --compact-steps 0 --strong-config none --cpu-seconds 0 > gpurun_out/r03b_launches_$i.log 2> gpurun_out/r03b_launches_$i.err || { tail -20 gpurun_out/r03b_launches_$i.err; exit 1; }
  tail -1 gpurun_out/r03b_launches_$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; a=d['raster_autotune']
print(round(d['value']/1e6,3), r['kernel'], round(r['kernel_ms'],4), 'fused', a['fused'].get('chosen'), a['fused'].get('recheck'), 'slots', a['ring']['repair'][-1]['slot_ms'])"
  grep -v amdgpu.ids gpurun_out/r03b_launches_$i.err | tail -25 | tr '\n' ' '; echo
done
