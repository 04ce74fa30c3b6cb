#!/bin/bash
# C4: the whole 65,536-env workload on one GPU, and one rank's shard of the 8-GPU split (8,192 envs).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/c4
for n in 65536 8192 8192; do
  timeout -k 10 300 python3 $R/bench.py --config C4 --envs $n --steps 100 --warmup 10 --cpu-seconds 0 --compact-steps 0 > $R/gpurun_out/c4/b$n.log 2>&1 || exit 1
  grep '^{' $R/gpurun_out/c4/b$n.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); r = d['roofline']; a = d['raster_autotune']; g = a.get('ring', {})
print('C4 n=$n', round(d['value'] / 1e6, 2), 'M', round(d['ms_per_step'], 4), r['kernel'], round(r['kernel_ms'], 4), round(r['frac'], 3),
      g.get('pair_gbs_min'), g.get('pair_gbs_max'), g.get('partner_tries'), g.get('rebuilds'), g.get('reverts'))" || exit 1
done
