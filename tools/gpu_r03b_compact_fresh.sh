#!/bin/bash
# round 3 (second session): the compact layout as the only workload of a fresh process (no float32
# instance before it), three fresh processes; then the compact raster shapes once more
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --obs-format u8f16 --strong-config none --cpu-seconds 0 --steps 100 --warmup 10 > gpurun_out/r03b_compact_fresh_$i.log 2>&1 || { tail -20 gpurun_out/r03b_compact_fresh_$i.log; exit 1; }
  tail -1 gpurun_out/r03b_compact_fresh_$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; a=d['raster_autotune']
print('u8f16', round(d['value']/1e6,2), 'M', r['kernel'], round(r['kernel_ms'],4), round(r['frac'],3), a.get('shape_newest'), a.get('fused', {}).get('chosen'), a.get('fused', {}).get('flags'), a.get('fused', {}).get('recheck'), {k: a.get('ring', {}).get(k) for k in ('pair_probes','pair_gbs_min','pair_gbs_max','partner_tries')})"
done
