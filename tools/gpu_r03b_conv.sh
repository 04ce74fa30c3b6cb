#!/bin/bash
# round 3 (second session): the learner's MFMA convolutions (tools/conv_variants.py) + their parity tests
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/conv_variants.py 256 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r03b_conv_variants.txt || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_conv_mfma.py > gpurun_out/r03b_conv_tests.log 2>&1 || { tail -5 gpurun_out/r03b_conv_tests.log; grep -E "^E " gpurun_out/r03b_conv_tests.log | head; exit 1; }
tail -1 gpurun_out/r03b_conv_tests.log
