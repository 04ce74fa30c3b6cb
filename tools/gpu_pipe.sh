#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > /dev/null 2>&1 || exit 1
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -x -k "pipelined or step_parity" 2>&1 | tail -3 || exit 1
for cfg in C3; do for p in 1 2 4 1; do
  timeout -k 10 300 python bench.py --config $cfg --steps 100 --warmup 10 --cpu-seconds 0 --pipeline $p > gpurun_out/pipe_${cfg}_$p.log 2>&1 || exit 1
  python -c "import json;d=json.loads([l for l in open('gpurun_out/pipe_${cfg}_$p.log') if l.startswith('{')][0]);print('$cfg pipeline=$p', '%.3e'%d['value'], 'step_ms_ev %.3f'%d['step_ms_events'], 'raster/step %.3f'%d['raster_ms_per_step'], 'GB/s %.0f'%d['roofline']['achieved'], d['raster_autotune'])"
done; done
