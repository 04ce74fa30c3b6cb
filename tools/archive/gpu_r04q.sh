#!/bin/bash
# round 4: conv forward B-fragment prefetch (FFMP_CONV_BAHEAD 1 / 2) and forward occupancy (2 / 1
# workgroups per CU): conv parity with each variant library, then the conv2 kernels at B = 256
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04q
mkdir -p $O
for v in b2 b2o1; do
  FFMP_LIB=$R/tools/_build/libffmp_$v.so timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_conv_mfma.py -x -q --timeout 200 --timeout-method thread > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v conv parity: $(tail -1 $O/pytest_$v.log)"
done
for rep in 0 1; do
  for v in b1 b2 b2o1; do
    echo "== $v"
    FFMP_LIB=$R/tools/_build/libffmp_$v.so timeout -k 10 300 python $R/tools/conv_probe.py 256 --mfma-only 2>&1 | grep mfma || exit 1
  done
done
