#!/bin/bash
# env kernel by lanes per env and waves per block with the chunked lidar (ch3 = default build, ch2)
# builds first, on the CPU: for ch in 1 2 3 4 6: hipcc (the Makefile's HIPFLAGS) -DFFMP_BEAM_CHUNK=$ch
#   -o tools/_build/libffmp_ch$ch.so <the three csrc/*.hip>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
B=$R/tools/_build
for rep in 0 1; do
  for ch in 3 2; do
    for l in 16 32 64; do
      for w in 1 4; do
        FFMP_ENV_LANES=$l FFMP_ENV_WAVES=$w FFMP_LIB=$B/libffmp_ch$ch.so timeout -k 10 200 python3 $R/tools/env_kernel_breakdown.py --preset C3 --envs 32768 base 2>&1 | grep 'env kernel' | sed "s/^/ch$ch lanes $l waves $w /" || exit 1
      done
    done
  done
done
for l in 32 64; do
  FFMP_ENV_LANES=$l FFMP_LIB=$B/libffmp_ch3.so timeout -k 10 200 python3 $R/tools/env_kernel_breakdown.py --preset C5 --envs 16384 base 2>&1 | grep 'env kernel' | sed "s/^/ch3 lanes $l /" || exit 1
done
