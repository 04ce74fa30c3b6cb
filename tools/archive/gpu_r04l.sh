#!/bin/bash
# round 4: the 32 -> 64 weight gradient with 8 taps per wave (tools/_build/libffmp_tw8.so: the Makefile's
# HIPFLAGS + -DFFMP_WGRAD_TW_3264=8; 1 wave per SIMD) against the shipped 4: parity, then timing by chunks
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04l
mkdir -p $O
FFMP_LIB=$R/tools/_build/libffmp_tw8.so timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_conv_mfma.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_tw8.log 2>&1 || { tail -30 $O/pytest_tw8.log; exit 1; }
echo "tw8 parity: $(tail -1 $O/pytest_tw8.log)"
for rep in 0 1; do
  timeout -k 10 200 python $R/tools/wgrad_probe.py 4 8 16 32 2>&1 | grep wgrad | sed "s/^/tw4 /" || exit 1
  FFMP_LIB=$R/tools/_build/libffmp_tw8.so timeout -k 10 200 python $R/tools/wgrad_probe.py 4 8 16 32 2>&1 | grep wgrad | sed "s/^/tw8 /" || exit 1
done
