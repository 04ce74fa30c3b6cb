#!/bin/bash
# env-step latency chain change: GPU parity suite, the in-kernel trace, C2 / C3 benches.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/pytest_gpu.log 2>&1 || { tail -30 $R/gpurun_out/pytest_gpu.log; exit 1; }
tail -2 $R/gpurun_out/pytest_gpu.log
bash $R/tools/gpu_trace.sh > $R/gpurun_out/trace.log 2>&1 || exit 1
for F in off on; do
  timeout -k 10 200 python3 $R/bench.py --config C2 --fused $F --steps 200 --warmup 20 --cpu-seconds 0 > $R/gpurun_out/c2_$F.log 2>&1 || exit 1
  grep '^{' $R/gpurun_out/c2_$F.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('C2 fused=$F', round(d['value']/1e6,2), 'M', round(d['ms_per_step'],4), round(r['kernel_ms'],4), r['kernel'], round(r['frac'],3))" || exit 1
done
timeout -k 10 200 python3 $R/tools/env_kernel_breakdown.py --preset C3 --envs 32768 base "L=0 (no lidar)" "no resets" 2>&1 | grep 'env kernel' || exit 1
timeout -k 10 200 python3 $R/tools/env_kernel_breakdown.py --preset C2 --envs 4096 base "no resets" 2>&1 | grep 'env kernel' || exit 1
timeout -k 10 300 python3 $R/bench.py --steps 100 --warmup 20 --cpu-seconds 0 > $R/gpurun_out/c3.log 2>&1 || exit 1
grep '^{' $R/gpurun_out/c3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('C3', round(d['value']/1e6,2), 'M', round(d['ms_per_step'],4), round(r['kernel_ms'],4), r['kernel'], round(r['frac'],3), d['raster_autotune']['fused'])"
