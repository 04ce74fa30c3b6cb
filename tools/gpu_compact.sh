#!/bin/bash
# compact observation format: GPU tests (new + full suite), then C3/C2/C5 bench lines of both formats
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > /dev/null 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_compact.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_compact.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_compact.log
[ $rc -eq 0 ] || exit $rc
if [ "${FULL:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  tail -3 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
fi
[ $# -gt 0 ] || set -- "C3 u8f16" "C3 f32"
for spec in "$@"; do
  set -- $spec
  timeout -k 10 300 python bench.py --config $1 --obs-format $2 --steps 100 --warmup 10 --cpu-seconds 0 > gpurun_out/compact_$1_$2.log 2>&1 || { tail -5 gpurun_out/compact_$1_$2.log; exit 1; }
  python -c "import json;d=json.loads([l for l in open('gpurun_out/compact_$1_$2.log') if l.startswith('{')][0]);print('$1 $2', '%.3e'%d['value'], 'step_ms_ev %.3f'%d['step_ms_events'], 'kernel/step %.3f'%d['raster_ms_per_step'], 'GB/s %.0f'%d['roofline']['achieved'], d['roofline']['kernel'], d['raster_autotune']['shape'], d['raster_autotune'].get('gbs'), (d['raster_autotune'].get('fused') or {}).get('chosen'))"
done
