#!/bin/bash
# env kernel at the fewest lanes per env (the new auto rule) by beams per chunk (ch3 = default build)
# builds first, on the CPU: for ch in 1 2 3 4 6: hipcc (the Makefile's HIPFLAGS) -DFFMP_BEAM_CHUNK=$ch
#   -o tools/_build/libffmp_ch$ch.so <the three csrc/*.hip>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
B=$R/tools/_build
for rep in 0 1; do
  for ch in 3 4 6; do
    FFMP_LIB=$B/libffmp_ch$ch.so timeout -k 10 200 python3 $R/tools/env_kernel_breakdown.py --preset C3 --envs 32768 base 2>&1 | grep 'env kernel' | sed "s/^/ch$ch auto lanes /" || exit 1
    FFMP_LIB=$B/libffmp_ch$ch.so timeout -k 10 200 python3 $R/tools/env_kernel_breakdown.py --preset C5 --envs 16384 base 2>&1 | grep 'env kernel' | sed "s/^/ch$ch auto lanes /" || exit 1
  done
done
