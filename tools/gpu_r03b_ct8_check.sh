#!/bin/bash
# round 3 (second session): the 8-cells-per-lane compact raster: parity, then the default bench twice
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_timed_path.py tests/test_gpu_compact.py tests/test_gpu_oracle_c.py > gpurun_out/r03b_ct8_tests.log 2>&1 || { tail -5 gpurun_out/r03b_ct8_tests.log; grep -E "^E " gpurun_out/r03b_ct8_tests.log | head -20; exit 1; }
tail -1 gpurun_out/r03b_ct8_tests.log
for i in 1 2; do
  timeout -k 10 400 python -u bench.py > gpurun_out/r03b_ct8_bench_$i.log 2>&1 || { tail -20 gpurun_out/r03b_ct8_bench_$i.log; exit 1; }
  tail -1 gpurun_out/r03b_ct8_bench_$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['compact_layout']; r=d['roofline']
print('f32', round(d['value']/1e6,3), r['kernel'], round(r['kernel_ms'],4), round(r['frac'],3), '| compact', round(c['value']/1e6,2), c['kernel'], round(c['kernel_ms'],4), round(c['frac'],3), c['shape'], c['fused'])"
done
