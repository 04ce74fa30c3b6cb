#!/bin/bash
# Seamless frame ring on the box: all GPU tests (seamless is the default ring), bench A/B (seamless vs wrap).
set -o pipefail
mkdir -p gpurun_out
echo "== gpu tests"; timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/ring_tests.log 2>&1; rc=$?
tail -5 gpurun_out/ring_tests.log; [ $rc -eq 0 ] || exit $rc
for ring in seamless wrap seamless; do
  echo "== bench $ring"; timeout -k 10 300 python bench.py --ring $ring --steps 100 --warmup 10 --cpu-seconds 0 > gpurun_out/bench_$ring.log 2>&1 || exit 1
  python -c "import json;d=json.loads([l for l in open('gpurun_out/bench_$ring.log') if l.startswith('{')][0]);r=d['roofline'];print('$ring', d['config']['ring'], '%.4e'%d['value'], 'raster %.3f ms'%r['kernel_ms'], '%.0f GB/s'%r['achieved'], 'full', r['full_launches'], 'tries', d['raster_autotune'].get('placement_tries'))"
done
