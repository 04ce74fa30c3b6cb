#!/bin/bash
# env kernel alone vs its occupancy bound (__launch_bounds__ min waves per SIMD 5 / 6 / 8, with
# scratch spills) against the in-tree build (119 VGPRs, 4 waves)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for v in tree w5 w6 w8 tree; do
  if [ $v = tree ]; then L=$R/flow_field_based_motion_planner_amd/lib/libffmp.so; else L=$R/tools/_build/libffmp_$v.so; fi
  FFMP_LIB=$L timeout -k 10 200 python3 $R/tools/env_kernel_breakdown.py --preset C3 --envs 32768 base 2>&1 | grep 'env kernel' | sed "s/^/$v /" || exit 1
  FFMP_LIB=$L timeout -k 10 200 python3 $R/tools/env_kernel_breakdown.py --preset C5 --envs 16384 base 2>&1 | grep 'env kernel' | sed "s/^/$v /" || exit 1
done
