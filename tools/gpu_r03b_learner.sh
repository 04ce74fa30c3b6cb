#!/bin/bash
# round 3 (second session): learner tests + the train.py-style loop on the current MFMA kernels
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_learner.py tests/test_gpu_conv_mfma.py > gpurun_out/r03b_learner_tests.log 2>&1 || { tail -5 gpurun_out/r03b_learner_tests.log; grep -E "^E " gpurun_out/r03b_learner_tests.log | head; exit 1; }
tail -1 gpurun_out/r03b_learner_tests.log
for i in 1 2; do
  timeout -k 10 300 python -u examples/train_vec.py --envs 256 --steps 100 --amp > gpurun_out/r03b_train_vec_amp_$i.log 2>&1 || { tail -20 gpurun_out/r03b_train_vec_amp_$i.log; exit 1; }
  tail -1 gpurun_out/r03b_train_vec_amp_$i.log | cut -c1-200
done
timeout -k 10 300 python -u examples/train_vec.py --envs 256 --steps 100 --amp --temporal-maps --input-channels 3 > gpurun_out/r03b_train_vec_tm3.log 2>&1 || { tail -20 gpurun_out/r03b_train_vec_tm3.log; exit 1; }
tail -1 gpurun_out/r03b_train_vec_tm3.log | cut -c1-300
