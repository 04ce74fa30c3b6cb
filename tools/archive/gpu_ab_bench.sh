#!/bin/bash
# A/B of two libffmp builds by whole bench.py runs (f32 metric + compact_layout), alternating fresh
# processes: tools/_build/libffmp_base.so (before) vs the in-tree lib (after).  usage: [reps] [config]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/ab
for rep in $(seq 1 ${1:-3}); do
  for v in base new; do
    if [ $v = base ]; then L=$R/tools/_build/libffmp_base.so; else L=$R/flow_field_based_motion_planner_amd/lib/libffmp.so; fi
    FFMP_LIB=$L timeout -k 10 300 python3 $R/bench.py --config ${2:-C3} --steps 50 --warmup 10 --cpu-seconds 0 > $R/gpurun_out/ab/b_${v}_$rep.log 2>&1 || exit 1
    grep '^{' $R/gpurun_out/ab/b_${v}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; c=d.get('compact_layout') or {}; a=d['raster_autotune']; print('$v', d['config']['workload'], 'f32', round(d['value']/1e6,2), 'M', r['kernel'], round(r['kernel_ms'],4), {k: a.get('ring', {}).get(k) for k in ('pair_probes', 'pair_gbs_min', 'pair_gbs_max')}, '| compact', round(c.get('value', 0)/1e6,2), 'M', round(c.get('kernel_ms', 0),4), c.get('shape'), c.get('ring_pairing'))" || exit 1
  done
done
