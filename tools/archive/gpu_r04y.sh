#!/bin/bash
# round 4: conv3 / conv4 forwards per shape: conv_small_kernel (default: up to 2,048 positions) against
# the row-ring conv_fwd_kernel (FFMP_CONV_SMALL_MAX lowered: a probe build, tools/_build/libffmp_sm.so,
# whose launch_fwd reads that variable; the shipped routing is unchanged), B = 256
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for rep in 0 1; do
  for m in 2048 600 300 0; do
    FFMP_LIB=$R/tools/_build/libffmp_sm.so FFMP_CONV_SMALL_MAX=$m timeout -k 10 120 python $R/tools/conv_small_probe.py || exit 1
  done
done
