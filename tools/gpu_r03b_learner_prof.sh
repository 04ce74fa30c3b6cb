#!/bin/bash
# round 3 (second session): kernel split of the train.py-style loop on the current MFMA kernels, then
# the default bench as the driver runs it
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train2 -o train -- python3 examples/train_vec.py --envs 256 --steps 60 --amp > gpurun_out/r03b_train_prof.log 2>&1 || { tail -20 gpurun_out/r03b_train_prof.log; exit 1; }
tail -1 gpurun_out/r03b_train_prof.log
timeout -k 10 400 python -u bench.py > gpurun_out/r03b_bench_default.log 2>&1 || { tail -20 gpurun_out/r03b_bench_default.log; exit 1; }
tail -1 gpurun_out/r03b_bench_default.log | cut -c1-600
