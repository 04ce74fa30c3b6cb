#!/bin/bash
# round 3 (second session): the one-launch step rastering from the speculative record (the env wave
# joins the raster after the lidar / reward / reset work): parity, then A/B against the previous build
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/ab
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_timed_path.py tests/test_gpu_parity.py tests/test_gpu_compact.py tests/test_gpu_oracle_c.py > gpurun_out/r03b_spec_tests.log 2>&1 || { tail -5 gpurun_out/r03b_spec_tests.log; grep -E "^E " gpurun_out/r03b_spec_tests.log | head -20; exit 1; }
tail -2 gpurun_out/r03b_spec_tests.log
for rep in 1 2; do
  for v in base new; do
    if [ $v = base ]; then L=$R/tools/_build/libffmp_base.so; else L=$R/flow_field_based_motion_planner_amd/lib/libffmp.so; fi
    FFMP_LIB=$L timeout -k 10 300 python3 $R/bench.py --steps 50 --warmup 10 --cpu-seconds 0 > $R/gpurun_out/ab/s_${v}_$rep.log 2>&1 || exit 1
    grep '^{' $R/gpurun_out/ab/s_${v}_$rep.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; c=d.get('compact_layout') or {}; f=d['raster_autotune'].get('fused', {})
print('$v', 'f32', round(d['value']/1e6,3), 'M', r['kernel'], round(r['kernel_ms'],4), 'fused', f.get('chosen'), f.get('recheck'), 'slots', d['raster_autotune'].get('ring', {}).get('repair', [{}])[-1].get('slot_ms'), '| compact', round(c.get('value', 0)/1e6,2), 'M', c.get('kernel'), round(c.get('kernel_ms', 0),4), c.get('fused'))" || exit 1
  done
done
