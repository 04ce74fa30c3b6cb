#!/bin/bash
# round 4, final code: the full GPU suite + smoke, rocprofv3 trace + PMC of the C3 bench, the driver's
# bench line twice, C2 and the C5 share
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04j
mkdir -p $O
export FFMP_TIMED_PATH_OUT=$O
timeout -k 10 900 python -u -m pytest -x -v --timeout 900 --timeout-method thread $R/tests -m gpu > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
rm -rf $R/gpurun_out/prof
bash $R/tools/gpu_profile.sh r04 C3 > $O/profile.log 2>&1 || { tail -30 $O/profile.log; exit 1; }
for rep in 0 1; do
  timeout -k 10 400 python $R/bench.py --steps 20 --warmup 5 > $O/bench_default$rep.json 2> $O/bench_default$rep.err || exit 1
  python -c "import json; d=json.loads(open('$O/bench_default$rep.json').read().strip().splitlines()[-1]); print('default', round(d['value']/1e6,3), round(d['roofline']['kernel_ms'],4), round(d['roofline']['frac'],4), round(d['hbm_roofline_pct_whole_step'],2), round(d['compact_layout']['value']/1e6,3), round(d['strong']['value']/1e6,3))"
done
timeout -k 10 300 python $R/bench.py --config C2 --steps 200 --warmup 20 --strong-config none --compact-steps 0 --cpu-seconds 0 > $O/bench_c2.json 2>/dev/null || exit 1
timeout -k 10 400 python $R/bench.py --config C5 --steps 30 --warmup 5 --strong-config none --compact-steps 0 --cpu-seconds 0 > $O/bench_c5.json 2>/dev/null || exit 1
for c in c2 c5; do python -c "import json; d=json.loads(open('$O/bench_$c.json').read().strip().splitlines()[-1]); print('$c', d['config']['n_envs_per_gpu'], round(d['value']/1e6,3), round(d['roofline']['kernel_ms'],4), round(d['roofline']['frac'],4), round(d['hbm_roofline_pct_whole_step'],2))"; done
