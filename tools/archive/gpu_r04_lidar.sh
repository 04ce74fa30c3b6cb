#!/bin/bash
# round 4: the env kernel's lidar with deferred square roots (FFMP_LIDAR_DEFER) and the env's outputs
# written before its lidar (env_group restructure), beams per chunk.
# Builds (CPU, tools/_build): hipcc (the Makefile's HIPFLAGS) -DFFMP_BEAM_CHUNK=ch -DFFMP_LIDAR_DEFER=d
#   -c ffmp_kernels.hip, linked with ffmp_ring.o + ffmp_conv.o into libffmp_<V>.so:
#   A = round-3 env_group, ch3 d0;  N = round-4 env_group ch3 d0;  P = ch3 d1;  Q = ch2 d1
# parity (whole-config C oracle + step parity) with P, then the env kernel alone, alternating builds.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_lidar
mkdir -p $O
B=$R/tools/_build
for v in P; do
  FFMP_LIB=$B/libffmp_$v.so timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_oracle_c.py $R/tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v parity: $(tail -1 $O/pytest_$v.log)"
done
for rep in 0 1; do
  for v in A N P Q; do
    FFMP_LIB=$B/libffmp_$v.so timeout -k 10 200 python3 $R/tools/env_kernel_breakdown.py --preset C3 --envs 32768 base "L=0 (no lidar)" 2>&1 | grep 'env kernel' | sed "s/^/$v /" || exit 1
  done
done
for v in A N P Q; do
  FFMP_LIB=$B/libffmp_$v.so timeout -k 10 200 python3 $R/tools/env_kernel_breakdown.py --preset C5 --envs 16384 base 2>&1 | grep 'env kernel' | sed "s/^/$v /" || exit 1
done
