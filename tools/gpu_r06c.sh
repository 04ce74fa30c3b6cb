#!/bin/bash
# round 6 (c): conv launch variants (MFMA shape, kernel rows per ring step, B through LDS): parity + A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06c
mkdir -p $O
cd $R
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv_mfma.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_conv.log 2>&1; rc=$?
tail -3 $O/pytest_conv.log; grep -E "^FAILED|Error" $O/pytest_conv.log | head -20; ok $rc || exit 1
timeout -k 10 300 python -u tools/conv_ab.py 256 7 0:0:0 32:1:0 32:1:1 32:4:0 > $O/conv_ab.txt 2>&1 || { tail -20 $O/conv_ab.txt; exit 1; }
cat $O/conv_ab.txt
