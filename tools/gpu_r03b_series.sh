#!/bin/bash
# round 3 (second session): k-frame temporal maps (env, replay, Brain, 3-channel conv1 fold), then the
# learner's kernel split, then the default bench as the driver runs it
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_temporal_maps.py tests/test_gpu_replay.py tests/test_gpu_learner.py "tests/test_gpu_conv_mfma.py::test_folded_conv1_against_float64" > gpurun_out/r03b_series_tests.log 2>&1 || { tail -5 gpurun_out/r03b_series_tests.log; grep -E "^E " gpurun_out/r03b_series_tests.log | head -20; exit 1; }
tail -2 gpurun_out/r03b_series_tests.log
bash tools/gpu_r03b_learner_prof.sh
