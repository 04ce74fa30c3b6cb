#!/bin/bash
# round 4: the weight gradient with its operand reads one k-step ahead (FFMP_WGRAD_PREFETCH, the
# 32 -> 64 kernel): conv parity with that library, then the conv2 kernels at B = 256 with / without
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04s
mkdir -p $O
FFMP_LIB=$R/tools/_build/libffmp_wpa.so timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_conv_mfma.py $R/tests/test_gpu_learner.py -x -q --timeout 200 --timeout-method thread > $O/pytest_wpa.log 2>&1 || { tail -30 $O/pytest_wpa.log; exit 1; }
echo "wpa conv + learner parity: $(tail -1 $O/pytest_wpa.log)"
for rep in 0 1; do
  for v in wp0 wpa; do
    echo "== $v"
    FFMP_LIB=$R/tools/_build/libffmp_$v.so timeout -k 10 300 python $R/tools/conv_probe.py 256 --mfma-only 2>&1 | grep mfma || exit 1
  done
done
