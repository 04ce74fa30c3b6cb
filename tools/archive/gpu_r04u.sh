#!/bin/bash
# round 4: conv forward with the next tap's B loads kept ahead of the MFMAs (a probe build with a
# scheduling barrier after load_b, -DFFMP_CONV_BFIRST=1; not kept, so not in the source any more):
# conv parity with that library, then the conv2 kernels at B = 256 against the current one
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04u
mkdir -p $O
FFMP_LIB=$R/tools/_build/libffmp_bf.so timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_conv_mfma.py -x -q --timeout 200 --timeout-method thread > $O/pytest_bf.log 2>&1 || { tail -30 $O/pytest_bf.log; exit 1; }
echo "bf conv parity: $(tail -1 $O/pytest_bf.log)"
for rep in 0 1; do
  for v in cur bf; do
    echo "== $v"
    FFMP_LIB=$R/tools/_build/libffmp_$v.so timeout -k 10 300 python $R/tools/conv_probe.py 256 --mfma-only 2>&1 | grep mfma || exit 1
  done
done
