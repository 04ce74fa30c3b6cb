#!/bin/bash
# C2 raster rate by frame layout: seamless VMM ring (default), wrapping ring in the arena,
# contiguous W = 2; two alternating rounds.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/c2l
for rep in 1 2; do
  for lay in "--ring seamless" "--ring wrap" "--frame-window 2"; do
    timeout -k 10 200 python3 $R/bench.py --config C2 $lay --steps 100 --warmup 10 --cpu-seconds 0 --compact-steps 0 > $R/gpurun_out/c2l/b.log 2>&1 || exit 1
    grep '^{' $R/gpurun_out/c2l/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$lay', round(d['value']/1e6,2), 'M', r['kernel'], round(r['kernel_ms'],4), round(r['achieved']), 'GB/s', 'full', r['full_launches'], d['config']['frame_window'], d['config']['ring'])" || exit 1
  done
done
