#!/bin/bash
# env kernel alone at C3 / C5 for diagnostic builds of the lidar (tools/_build/libffmp_<v>.so)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for v in base ${@}; do
  if [ $v = base ]; then L=$R/flow_field_based_motion_planner_amd/lib/libffmp.so; else L=$R/tools/_build/libffmp_$v.so; fi
  FFMP_LIB=$L timeout -k 10 200 python3 $R/tools/env_kernel_breakdown.py --preset C3 --envs 32768 base "L=0 (no lidar)" 2>&1 | grep 'env kernel' | sed "s/^/$v /" || exit 1
done
