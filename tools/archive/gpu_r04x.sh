#!/bin/bash
# round 4: the conv forward kernel compiled for 3 workgroups per CU (FFMP_CONV_FWD_OCC=3: the data
# gradient's ring leaves LDS room for three) against 2: conv parity, then the conv2 kernels at B = 256
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04x
mkdir -p $O
FFMP_LIB=$R/tools/_build/libffmp_occ3.so timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_conv_mfma.py -x -q --timeout 200 --timeout-method thread > $O/pytest_occ3.log 2>&1 || { tail -30 $O/pytest_occ3.log; exit 1; }
echo "occ3 conv parity: $(tail -1 $O/pytest_occ3.log)"
for rep in 0 1; do
  for v in cur occ3; do
    echo "== $v"
    FFMP_LIB=$R/tools/_build/libffmp_$v.so timeout -k 10 300 python $R/tools/conv_probe.py 256 --mfma-only 2>&1 | grep mfma || exit 1
  done
done
