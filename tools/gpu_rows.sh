#!/bin/bash
# compact raster with row staging (FFMP_RASTER_ROWS): compact parity tests, then the compact C3
# bench twice (autotune candidates incl. ROWS shapes)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_compact.py -x -q --timeout 300 --timeout-method thread > gpurun_out/rows_pytest.log 2>&1 || { tail -30 gpurun_out/rows_pytest.log; exit 1; }
tail -2 gpurun_out/rows_pytest.log
for k in 1 2; do
  timeout -k 10 300 python bench.py --obs-format u8f16 --cpu-seconds 0 --steps 100 > gpurun_out/rows_bench$k.log 2>&1 || { tail -20 gpurun_out/rows_bench$k.log; exit 1; }
  python -c "
import json;d=json.loads([l for l in open('gpurun_out/rows_bench$k.log') if l.startswith('{')][0]);a=d['raster_autotune']
print('value %.4g step_ms %.4f raster_ms %.4f GB/s %.0f' % (d['value'], d['step_ms_events'], d['roofline']['kernel_ms'], d['roofline']['achieved']), a['shape'])
print(a.get('candidates'))"
done
