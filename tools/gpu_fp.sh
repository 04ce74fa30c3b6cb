#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/pytest_gpu.log 2>&1 || { tail -30 $R/gpurun_out/pytest_gpu.log; exit 1; }
tail -1 $R/gpurun_out/pytest_gpu.log
FFMP_LIB=$R/tools/_build/libffmp_trace.so timeout -k 10 300 python3 $R/tools/trace_probe.py C3 32768 fused 2>&1 | grep -v amdgpu.ids | head -15 || exit 1
for v in base new; do
  if [ $v = base ]; then L=$R/tools/_build/libffmp_base.so; else L=$R/flow_field_based_motion_planner_amd/lib/libffmp.so; fi
  FFMP_LIB=$L timeout -k 10 200 python3 $R/tools/env_kernel_breakdown.py --preset C2 --envs 4096 base 2>&1 | grep 'env kernel' | sed "s/^/$v /" || exit 1
  FFMP_LIB=$L timeout -k 10 200 python3 $R/tools/env_kernel_breakdown.py --preset C3 --envs 32768 base 2>&1 | grep 'env kernel' | sed "s/^/$v /" || exit 1
done
bash $R/tools/gpu_ab_bench.sh 2
