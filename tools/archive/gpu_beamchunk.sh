#!/bin/bash
# lidar beams traced CH at a time per lane (trace_beams, FFMP_BEAM_CHUNK): whole-config oracle
# builds first, on the CPU: for ch in 1 2 3 4 6: hipcc (the Makefile's HIPFLAGS) -DFFMP_BEAM_CHUNK=$ch
#   -o tools/_build/libffmp_ch$ch.so <the three csrc/*.hip>
# parity with each chunked build, then the env kernel alone, alternating builds (C3, C5, C2)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
B=$R/tools/_build
for ch in 2 3; do
  FFMP_LIB=$B/libffmp_ch$ch.so timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_oracle_c.py -m gpu -x -q --timeout 300 --timeout-method thread > $R/gpurun_out/bc_pytest_ch$ch.log 2>&1 || { tail -30 $R/gpurun_out/bc_pytest_ch$ch.log; exit 1; }
  echo "ch$ch parity: $(tail -1 $R/gpurun_out/bc_pytest_ch$ch.log)"
done
for rep in 0 1; do
  for ch in 1 2 3 4; do
    FFMP_LIB=$B/libffmp_ch$ch.so timeout -k 10 200 python3 $R/tools/env_kernel_breakdown.py --preset C3 --envs 32768 base 2>&1 | grep 'env kernel' | sed "s/^/ch$ch /" || exit 1
  done
done
for ch in 1 2 3; do
  FFMP_LIB=$B/libffmp_ch$ch.so timeout -k 10 200 python3 $R/tools/env_kernel_breakdown.py --preset C5 --envs 16384 base 2>&1 | grep 'env kernel' | sed "s/^/ch$ch /" || exit 1
done
