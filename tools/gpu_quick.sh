#!/bin/bash
# quick check: GPU parity tests + C3/C5 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > /dev/null 2>&1 || exit 1
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_quick.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_quick.log
[ $rc -eq 0 ] || exit $rc
for cfg in ${@:-C3}; do
  timeout -k 10 300 python bench.py --config $cfg --steps 100 --warmup 10 --cpu-seconds 0 > gpurun_out/quick_$cfg.log 2>&1 || exit 1
  python -c "import json;d=json.loads([l for l in open('gpurun_out/quick_$cfg.log') if l.startswith('{')][0]);print('$cfg', '%.3e'%d['value'], 'step_ms_ev %.3f'%d['step_ms_events'], 'raster/step %.3f'%d['raster_ms_per_step'], 'GB/s %.0f'%d['roofline']['achieved'], d['raster_autotune'])"
done
