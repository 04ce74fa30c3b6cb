#!/bin/bash
# round 3 (second session): the driver's bench command with the launch shape fixed to 4096-cell blocks
# (the shape with the post-idle slow start), per-launch raster times, three fresh processes
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup ${WARM:-5} --dump-launches --compact-steps 0 --strong-config none --cpu-seconds 0 --tuning tools/tuning_c3_4096x37.json > gpurun_out/r03b_loop_$i.log 2> gpurun_out/r03b_loop_$i.err || { tail -20 gpurun_out/r03b_loop_$i.err; exit 1; }
  tail -1 gpurun_out/r03b_loop_$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(round(d['value']/1e6,3), r['kernel'], round(r['kernel_ms'],4))"
  grep "raster ms" gpurun_out/r03b_loop_$i.err
done
