#!/bin/bash
# beam table in LDS: GPU parity suite, env kernel alone before (tools/_build/libffmp_base.so) / after,
# default bench and compact bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 900 python -u -m pytest $R/tests -m gpu -x -q --timeout 300 --timeout-method thread > $R/gpurun_out/pytest_gpu.log 2>&1 || { tail -30 $R/gpurun_out/pytest_gpu.log; exit 1; }
tail -1 $R/gpurun_out/pytest_gpu.log
for v in base new base new; do
  if [ $v = base ]; then L=$R/tools/_build/libffmp_base.so; else L=$R/flow_field_based_motion_planner_amd/lib/libffmp.so; fi
  FFMP_LIB=$L timeout -k 10 200 python3 $R/tools/env_kernel_breakdown.py --preset C3 --envs 32768 base 2>&1 | grep 'env kernel' | sed "s/^/$v /" || exit 1
  FFMP_LIB=$L timeout -k 10 200 python3 $R/tools/env_kernel_breakdown.py --preset C5 --envs 16384 base 2>&1 | grep 'env kernel' | sed "s/^/$v /" || exit 1
  FFMP_LIB=$L timeout -k 10 200 python3 $R/tools/env_kernel_breakdown.py --preset C2 --envs 4096 base 2>&1 | grep 'env kernel' | sed "s/^/$v /" || exit 1
done
for v in base new; do
  if [ $v = base ]; then L=$R/tools/_build/libffmp_base.so; else L=$R/flow_field_based_motion_planner_amd/lib/libffmp.so; fi
  FFMP_LIB=$L timeout -k 10 300 python bench.py --cpu-seconds 0 --compact-steps 100 > $R/gpurun_out/envb_$v.log 2>&1 || exit 1
  python -c "
import json;d=json.loads([l for l in open('$R/gpurun_out/envb_$v.log') if l.startswith('{')][0]);c=d['compact_layout']
print('$v C3 f32 %.4g step %.4f fused %s | compact %.4g step %.4f raster %.4f' % (d['value'], d['step_ms_events'], d['config']['fused'], c['value'], c['step_ms_events'], c['kernel_ms']))"
done
