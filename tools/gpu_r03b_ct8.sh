#!/bin/bash
# round 3 (second session): compact raster with 8 cells per lane (FFMP_RASTER_MID8): launch shapes at
# 6 (in-tree), 7 and 8 waves per SIMD (tools/_build/libffmp_ct8w*.so)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
for v in intree w7 w8; do
  if [ $v = intree ]; then L=$R/flow_field_based_motion_planner_amd/lib/libffmp.so; else L=$R/tools/_build/libffmp_ct8$v.so; fi
  echo "== $v"
  FFMP_LIB=$L timeout -k 10 300 python3 tools/compact_shapes.py C3 u8f16 2>&1 | grep -v amdgpu.ids || exit 1
done | tee gpurun_out/r03b_ct8_shapes2.txt
