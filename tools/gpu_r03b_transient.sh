#!/bin/bash
# round 3 (second session): the slow start of the timed loop (tools/transient_probe.py), two-launch step,
# with and without the constructor's settle cycles; then the driver's bench command twice
set -o pipefail
mkdir -p gpurun_out
for s in 0 1; do echo "== SETTLE=$s"; SETTLE=$s FUSED=off timeout -k 10 300 python3 tools/transient_probe.py 2>&1 | grep -v amdgpu.ids || exit 1; done | tee gpurun_out/r03b_transient3.txt
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --dump-launches --compact-steps 0 --strong-config none --cpu-seconds 0 > gpurun_out/r03b_settle_$i.log 2> gpurun_out/r03b_settle_$i.err || { tail -20 gpurun_out/r03b_settle_$i.err; exit 1; }
  tail -1 gpurun_out/r03b_settle_$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; a=d['raster_autotune']
print(round(d['value']/1e6,3), r['kernel'], round(r['kernel_ms'],4), 'fused', a['fused'].get('chosen'), a['fused'].get('recheck'), 'construct', d['construct_s'])"
  grep "raster ms" gpurun_out/r03b_settle_$i.err
done
