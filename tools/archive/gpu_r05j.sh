#!/bin/bash
# Round 5: where the compact raster's time goes — probe builds without the wall test, without the
# repulsive term, without the disc loop (outputs wrong; timing only), against the real kernel,
# on the shapes the autotune picks (32768/545, 65536/545), 3 alternating rounds.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05j
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for k in 1 2 3; do
  for v in real no_walls no_rep no_disc; do
    L=$R/tools/_probe/libffmp_$v.so
    [ $v = real ] && L=$R/flow_field_based_motion_planner_amd/lib/libffmp.so
    echo "== $v round $k"
    FFMP_LIB=$L timeout -k 10 180 python3 $R/tools/compact_shapes.py C3 u8f16 32768:545,65536:545,32768:545,65536:545 3 2>&1 | grep "rep 2" || exit 1
  done
done
