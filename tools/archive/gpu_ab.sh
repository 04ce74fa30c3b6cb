#!/bin/bash
# A/B of two libffmp builds on one box: tools/_build/libffmp_base.so (before) vs the in-tree lib
# (after), alternating fresh processes: compact C3 raster shapes and the default f32 bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/ab
for rep in 1 2; do
  for v in base new; do
    if [ $v = base ]; then L=$R/tools/_build/libffmp_base.so; else L=$R/flow_field_based_motion_planner_amd/lib/libffmp.so; fi
    echo "== $v rep $rep"
    FFMP_LIB=$L timeout -k 10 200 python3 $R/tools/compact_shapes.py C3 u8f16 2>&1 | grep "rep 1" || exit 1
    FFMP_LIB=$L timeout -k 10 300 python3 $R/bench.py --steps 50 --warmup 10 --cpu-seconds 0 > $R/gpurun_out/ab/b_${v}_$rep.log 2>&1 || exit 1
    grep '^{' $R/gpurun_out/ab/b_${v}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; c=d['compact_layout']; print('f32', round(d['value']/1e6,2), 'M', r['kernel'], round(r['kernel_ms'],4), '| compact', round(c['value']/1e6,2), 'M', round(c['kernel_ms'],4), c['shape'])" || exit 1
  done
done
