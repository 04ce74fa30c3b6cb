#!/bin/bash
# round 5 final evidence after the late learner changes (fragment-order weights, on-the-fly conv1 fold, fused Adam): the whole GPU suite, smoke(), the driver's command line twice, C2 at 200 steps twice,
# (final HEAD of round 5)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05final2
mkdir -p $O
export FFMP_TIMED_PATH_OUT=$O
cd $R && timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
for rep in 0 1; do
  timeout -k 10 400 python $R/bench.py --steps 20 --warmup 5 > $O/bench_default$rep.json 2> $O/bench_default$rep.err || { tail -20 $O/bench_default$rep.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_default$rep.json').read().strip().splitlines()[-1]); print('default', round(d['value']/1e6,3), round(d['roofline']['kernel_ms'],4), round(d['roofline']['frac'],4), round(d['hbm_roofline_pct_whole_step'],2), d['config']['graph'], round(d['compact_layout']['value']/1e6,3), round(d['compact_layout']['frac'],4), round(d['strong']['value']/1e6,3))"
done
for rep in 0 1; do
  timeout -k 10 400 python $R/bench.py --config C2 --steps 200 --warmup 20 > $O/bench_c2_$rep.json 2> $O/bench_c2_$rep.err || { tail -20 $O/bench_c2_$rep.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_c2_$rep.json').read().strip().splitlines()[-1]); print('C2', round(d['value']/1e6,3), round(d['ms_per_step']*1e3,1), 'us/step', round(d['roofline']['frac'],4), round(d['hbm_roofline_pct_whole_step'],2), d['config']['graph'])"
done
rm -rf $R/gpurun_out/prof
