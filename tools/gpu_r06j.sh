#!/bin/bash
# round 6 (j): conv A/B of the MFMA shape and tile for the folded conv1 and the rest (one process)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06j
mkdir -p $O
cd $R
timeout -k 10 400 python -u tools/conv_ab.py 256 9 0 32 > $O/conv_ab.txt 2>&1 || { tail -20 $O/conv_ab.txt; exit 1; }
cat $O/conv_ab.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv_mfma.py -q -m gpu --timeout 200 --timeout-method thread  2>&1 | tail -2
