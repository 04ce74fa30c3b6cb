#!/bin/bash
# round 6 (g): the whole GPU suite, smoke, and the driver's bench command line twice, on the final code
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06g
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log; grep -E "^FAILED" $O/pytest_gpu.log | head
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for rep in 1; do
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_default_$rep.json 2> $O/bench_default_$rep.err || { tail -20 $O/bench_default_$rep.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_default_$rep.json').read().strip().splitlines()[-1]); print('default', round(d['value']/1e6,3), round(d['roofline']['frac'],4), round(d['hbm_roofline_pct_whole_step'],2), d['cpu_baseline']['value'] if d.get('cpu_baseline') else None)"
done
