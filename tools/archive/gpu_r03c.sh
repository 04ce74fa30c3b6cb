#!/bin/bash
# Round 3, last session: GPU tasks.  usage: bash tools/gpu_r03c.sh <task>
#   full-bench   the whole -m gpu suite + smoke(), then the driver's bench command twice
#   prof         rocprofv3 kernel trace + stats of the bench (C3 legs, no CPU leg)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out

task_full() {
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03c_pytest_gpu.log 2>&1 || { tail -5 gpurun_out/r03c_pytest_gpu.log; grep -E "^E " gpurun_out/r03c_pytest_gpu.log | head -20; exit 1; }
  tail -1 gpurun_out/r03c_pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
}

task_bench() {
  for i in 1 2; do
    timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r03c_bench_$i.log 2>&1 || { tail -20 gpurun_out/r03c_bench_$i.log; exit 1; }
    tail -1 gpurun_out/r03c_bench_$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['compact_layout']; r=d['roofline']; s=d.get('strong') or {}; b=d['cpu_baseline']
print('f32', round(d['value']/1e6,3), 'step', round(d['ms_per_step'],4), r['kernel'], round(r['kernel_ms'],4), round(r['frac'],3), d['raster_autotune']['shape_newest'], '| strong', round(s.get('value',0)/1e6,3), '| compact', round(c['value']/1e6,2), round(c['step_ms_events'],4), round(c['kernel_ms'],4), round(c['frac'],3), c['shape'], '| cpu', round(b['value']/1e3,1), 'K')"
  done
}

task_prof() {
  rm -rf gpurun_out/prof_r03c
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r03c -o c3 -- python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/r03c_prof_bench.log 2>&1 || { tail -20 gpurun_out/r03c_prof_bench.log; exit 1; }
  f=$(find gpurun_out/prof_r03c -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/r03c_C3_final_kernel_stats.csv
  python3 -c "
import csv; rows=list(csv.DictReader(open('gpurun_out/r03c_C3_final_kernel_stats.csv')))
for r in rows[:8]: print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')"
  tail -1 gpurun_out/r03c_prof_bench.log | cut -c1-300
}

case "$1" in
  prof) task_prof ;;
  full-bench) task_full && task_bench ;;
  bench) task_bench ;;
  *) echo "usage: $0 {full-bench|bench|prof}"; exit 2 ;;
esac
