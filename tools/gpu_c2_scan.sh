#!/bin/bash
# C2 regime: raster rate vs env count at G = 128, and the env kernel's breakdown at C2.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/c2
for n in 4096 16384; do
  timeout -k 10 200 python3 $R/bench.py --config C2 --envs $n --fused off --steps 100 --warmup 10 --cpu-seconds 0 > $R/gpurun_out/c2/scan_$n.log 2>&1 || exit 1
  grep '^{' $R/gpurun_out/c2/scan_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('n=$n', round(d['value']/1e6,2), 'M', d['ms_per_step'], r['kernel_ms'], round(r['achieved']), d['raster_autotune'].get('shape_newest'), d['raster_autotune'].get('ring',{}).get('repair'))" || exit 1
done
timeout -k 10 200 python3 $R/tools/env_kernel_breakdown.py --preset C2 --envs 4096 base "K=0" "K=0,L=0,no collide" "no resets" "footprint only" 2>&1 | grep 'env kernel' || exit 1
timeout -k 10 200 python3 $R/tools/env_kernel_breakdown.py --preset C2 --envs 16384 base "no resets" 2>&1 | grep 'env kernel' || exit 1
