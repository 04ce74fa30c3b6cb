#!/bin/bash
# f32 C3 whole-step rate vs raster occupancy cap (dynamic LDS pad per block: 0 = 4 blocks/CU,
# 45000 B = 3, 60000 B = 2), alternating fresh bench.py processes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/occ
for rep in 1 2; do
  for pad in 0 45000 60000; do
    FFMP_RASTER_LDS_PAD=$pad timeout -k 10 300 python3 $R/bench.py --steps 50 --warmup 10 --cpu-seconds 0 --compact-steps 0 > $R/gpurun_out/occ/b_${pad}_$rep.log 2>&1 || exit 1
    grep '^{' $R/gpurun_out/occ/b_${pad}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; a=d['raster_autotune']; print('pad $pad', round(d['value']/1e6,2), 'M', r['kernel'], round(r['kernel_ms'],4), a['shape_newest'], a['fused'].get('two_launch_step_ms'), a['fused'].get('fused_step_ms'))" || exit 1
  done
done
