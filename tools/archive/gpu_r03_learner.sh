#!/bin/bash
# round 3: MFMA conv tests + learner tests, then the train.py-style loop with / without the MFMA convs,
# then a kernel-trace of the MFMA loop (per-kernel time split)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_conv_mfma.py tests/test_gpu_learner.py > gpurun_out/r03_conv_tests.log 2>&1 || { tail -5 gpurun_out/r03_conv_tests.log; grep -E "^E " gpurun_out/r03_conv_tests.log | head -8; exit 1; }
tail -2 gpurun_out/r03_conv_tests.log
timeout -k 10 300 python -u examples/train_vec.py --envs 256 --steps 100 --amp > gpurun_out/r03_train_vec_amp_mfma.log 2>&1 || { tail -20 gpurun_out/r03_train_vec_amp_mfma.log; exit 1; }
tail -1 gpurun_out/r03_train_vec_amp_mfma.log
timeout -k 10 400 python -u examples/train_vec.py --envs 256 --steps 100 --amp --no-mfma > gpurun_out/r03_train_vec_amp_miopen.log 2>&1 || { tail -20 gpurun_out/r03_train_vec_amp_miopen.log; exit 1; }
tail -1 gpurun_out/r03_train_vec_amp_miopen.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train -o train -- python3 examples/train_vec.py --envs 256 --steps 30 --amp > gpurun_out/r03_train_prof.log 2>&1 || { tail -20 gpurun_out/r03_train_prof.log; exit 1; }
find gpurun_out/prof_train -name "*stats*" | head
