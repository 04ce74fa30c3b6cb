#!/bin/bash
# round 4: data-gradient patch shapes BH x 32/BH (FFMP_DG_BH) with the step's A reads batched before
# its MFMAs, unconditionally (FFMP_DG_READS=1) or only for the blocks that compute (0):
# tools/_build/libffmp_dg<BH>r<READS>.so (the Makefile's HIPFLAGS + the two -D), against the row
# kernel (FFMP_CONV_DGRAD=0): parity, conv2 data-gradient timing at B = 256
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04f
mkdir -p $O
B=$R/tools/_build
V="1r1 2r1 4r1 2r0 4r0"
for v in $V; do
  FFMP_LIB=$B/libffmp_dg$v.so timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_conv_mfma.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_dg$v.log 2>&1 || { tail -30 $O/pytest_dg$v.log; exit 1; }
  echo "dg$v parity: $(tail -1 $O/pytest_dg$v.log)"
done
for rep in 0 1; do
  for v in $V; do
    FFMP_LIB=$B/libffmp_dg$v.so timeout -k 10 300 python $R/tools/conv_probe.py 256 2>&1 | grep "mfma dgrad" | sed "s/^/dg$v /" || exit 1
  done
  FFMP_CONV_DGRAD=0 timeout -k 10 300 python $R/tools/conv_probe.py 256 2>&1 | grep "mfma dgrad" | sed "s/^/rows /" || exit 1
done
