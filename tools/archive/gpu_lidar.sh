#!/bin/bash
# lidar beam-span culling: GPU parity suite, env-kernel timing before/after, benches.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/pytest_gpu.log 2>&1 || { tail -30 $R/gpurun_out/pytest_gpu.log; exit 1; }
tail -1 $R/gpurun_out/pytest_gpu.log
for v in base new; do
  if [ $v = base ]; then L=$R/tools/_build/libffmp_base.so; else L=$R/flow_field_based_motion_planner_amd/lib/libffmp.so; fi
  FFMP_LIB=$L timeout -k 10 200 python3 $R/tools/env_kernel_breakdown.py --preset C3 --envs 32768 base "L=0 (no lidar)" 2>&1 | grep 'env kernel' | sed "s/^/$v /" || exit 1
  FFMP_LIB=$L timeout -k 10 200 python3 $R/tools/env_kernel_breakdown.py --preset C5 --envs 16384 base "L=0 (no lidar)" 2>&1 | grep 'env kernel' | sed "s/^/$v /" || exit 1
done
bash $R/tools/gpu_ab_bench.sh 2 || exit 1
