#!/bin/bash
# the default bench workload three times in fresh processes on one box (spread of the metric)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/bench_spread.jsonl
for k in 1 2 3; do
  timeout -k 10 300 python bench.py --cpu-seconds 0 --compact-steps 0 > gpurun_out/bench_spread_$k.log 2>&1 || { tail -20 gpurun_out/bench_spread_$k.log; exit 1; }
  grep '^{' gpurun_out/bench_spread_$k.log >> gpurun_out/bench_spread.jsonl
  python -c "
import json;d=json.loads(open('gpurun_out/bench_spread.jsonl').read().splitlines()[-1])
print('run $k: %.4g env-steps/s, step %.4f ms, %s %.4f ms, frac %.3f' % (d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['kernel_ms'], d['roofline']['frac']))"
done
