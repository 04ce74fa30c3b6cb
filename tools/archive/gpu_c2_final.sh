#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/c2f
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/pytest_gpu.log 2>&1 || { tail -30 $R/gpurun_out/pytest_gpu.log; exit 1; }
tail -1 $R/gpurun_out/pytest_gpu.log
for rep in 1 2 3 4; do
  timeout -k 10 200 python3 $R/bench.py --config C2 --steps 200 --warmup 20 --cpu-seconds 0 --compact-steps 0 > $R/gpurun_out/c2f/b$rep.log 2>&1 || exit 1
  grep '^{' $R/gpurun_out/c2f/b$rep.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); r = d['roofline']; g = d['raster_autotune'].get('ring', {})
print('C2', round(d['value'] / 1e6, 2), 'M', r['kernel'], round(r['kernel_ms'], 4), round(r['achieved']), 'GB/s',
      g.get('pair_gbs_min'), g.get('pair_gbs_max'), g.get('partner_tries'), [x.get('slot_ms') for x in g.get('repair', [])],
      g.get('reverts'))" || exit 1
done
