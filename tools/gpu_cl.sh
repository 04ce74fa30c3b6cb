#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for f in "--amp --channels-last" "--channels-last"; do
timeout -k 10 400 python -u examples/train_vec.py --envs 256 --steps 60 $f > gpurun_out/train_vec_cl.log 2>&1 || { tail -20 gpurun_out/train_vec_cl.log; exit 1; }
grep '^{' gpurun_out/train_vec_cl.log | cut -c1-200
done
