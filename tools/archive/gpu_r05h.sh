#!/bin/bash
# round 5: the bench's graph-replay timed loop: graph parity, the full-size timed path (incl. graph replays),
# the driver's command line twice, and the rocprofv3 trace + PMC of the C3 bench (profiles/r05_C3_*)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05h
mkdir -p $O
export FFMP_TIMED_PATH_OUT=$O
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread $R/tests/test_gpu_graph.py $R/tests/test_gpu_timed_path.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 0 1; do
  timeout -k 10 400 python $R/bench.py --steps 20 --warmup 5 > $O/bench_default$rep.json 2> $O/bench_default$rep.err || { tail -20 $O/bench_default$rep.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_default$rep.json').read().strip().splitlines()[-1]); print('default', round(d['value']/1e6,3), round(d['roofline']['kernel_ms'],4), round(d['roofline']['frac'],4), round(d['hbm_roofline_pct_whole_step'],2), d['config']['graph'], round(d['compact_layout']['value']/1e6,3), round(d['compact_layout']['frac'],4), round(d['strong']['value']/1e6,3))"
done
rm -rf $R/gpurun_out/prof
bash $R/tools/gpu_profile.sh r05 C3 > $O/profile.log 2>&1 || { tail -30 $O/profile.log; exit 1; }
tail -30 $O/profile.log
