#!/bin/bash
# Round 5 (late): where conv_small_kernel's time goes (the Network's conv3 / conv4 forwards, B = 256) —
# probe builds (outputs wrong; timing only): nob = B fragments of tap 0 only (no per-tap weight
# loads), noepi = the 4 waves' partials not summed in the epilogue, wfrag = B stored and read in fragment
# order (every load instruction 1 KiB contiguous; outputs right); against the real kernel, 2 rounds.
# usage: gpu_r05sm.sh [variants...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05sm
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for k in 1 2; do
  for v in ${@:-real nob noepi}; do
    L=$R/tools/_probe/libffmp_sm$v.so
    [ $v = real ] && L=$R/flow_field_based_motion_planner_amd/lib/libffmp.so
    echo "== $v round $k"
    WF=; [ $v = wfrag ] && WF=1
    FFMP_SWEEP_WFRAG=$WF FFMP_LIB=$L FFMP_CONV_SMALL_MAX=$v timeout -k 10 120 python3 $R/tools/conv_small_probe.py 2>&1 | grep "small_max" || exit 1
  done
done
