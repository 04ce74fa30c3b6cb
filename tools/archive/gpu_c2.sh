#!/bin/bash
# C2 (4,096 envs, 128^2, 8 static discs) breakdown: two-launch vs one-launch step, kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/c2
cd /tmp && export TMPDIR=/tmp
for F in off on; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/c2/trace_$F -o run -- \
    python3 $R/bench.py --config C2 --fused $F --steps 200 --warmup 20 --cpu-seconds 0 > $R/gpurun_out/c2/bench_$F.log 2>&1 || exit 1
  find $R/gpurun_out/c2/trace_$F -name '*kernel_stats.csv' -exec cp {} $R/gpurun_out/c2/stats_$F.csv \;
  echo "== fused $F"; cut -c1-200 $R/gpurun_out/c2/stats_$F.csv | head -6
  grep '^{' $R/gpurun_out/c2/bench_$F.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['raster_autotune'].get('shape_newest'))"
done
