#!/bin/bash
# learner tests (incl. bf16 autocast) and the end-to-end training loop, fp32 vs --amp
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_learner.py tests/test_gpu_compact.py -x -q --timeout 200 --timeout-method thread > gpurun_out/amp_pytest.log 2>&1 || { tail -30 gpurun_out/amp_pytest.log; exit 1; }
tail -1 gpurun_out/amp_pytest.log
timeout -k 10 400 python -u examples/train_vec.py --envs 256 --steps 60 --amp > gpurun_out/train_vec_amp.log 2>&1 || { tail -20 gpurun_out/train_vec_amp.log; exit 1; }
grep '^{' gpurun_out/train_vec_amp.log | cut -c1-300
timeout -k 10 400 python -u examples/train_vec.py --envs 256 --steps 60 > gpurun_out/train_vec_fp32.log 2>&1 || { tail -20 gpurun_out/train_vec_fp32.log; exit 1; }
grep '^{' gpurun_out/train_vec_fp32.log | cut -c1-300
