#!/bin/bash
# Round 5: the skewed launch with its env blocks LAST where they outnumber the CUs (C3): graph tests (also with
# FFMP_SKEW_ENV_LAST=1 at the tests' small sizes), the full-size timed path (C3: env-last skewed replays), then
# C3 with --graph-skew on / off alternating twice and C2 (auto) once.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05y
mkdir -p $O
export FFMP_TIMED_PATH_OUT=$O
cd $R && timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_graph.py > $O/pytest_graph.log 2>&1 || { tail -30 $O/pytest_graph.log; exit 1; }
echo "graph tests: $(tail -1 $O/pytest_graph.log)"
FFMP_SKEW_ENV_LAST=1 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_graph.py -k skewed > $O/pytest_graph_last.log 2>&1 || { tail -30 $O/pytest_graph_last.log; exit 1; }
echo "graph tests, env last: $(tail -1 $O/pytest_graph_last.log)"
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 500 --timeout-method thread -m gpu tests/test_gpu_timed_path.py > $O/pytest_timed.log 2>&1 || { tail -30 $O/pytest_timed.log; exit 1; }
echo "timed path: $(tail -1 $O/pytest_timed.log)"
cd /tmp && export TMPDIR=/tmp
for k in 1 2; do
  for sk in on off; do
    timeout -k 10 300 python3 $R/bench.py --config C3 --graph-skew $sk --steps 96 --warmup 16 --cpu-seconds 0 --strong-config none --compact-steps 0 > $O/bench_C3_${sk}_$k.json 2> $O/bench_C3_${sk}_$k.err || { tail -20 $O/bench_C3_${sk}_$k.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/bench_C3_${sk}_$k.json').read().strip().splitlines()[-1]); r=d['roofline']; print('C3 skew $sk', round(d['value']/1e6,3), 'M', round(d['ms_per_step']*1e3,1), 'us/step', 'frac', round(r['frac'],4), round(d['hbm_roofline_pct_whole_step'],2))"
  done
done
timeout -k 10 300 python3 $R/bench.py --config C2 --steps 96 --warmup 16 --cpu-seconds 0 --strong-config none --compact-steps 0 > $O/bench_C2.json 2> $O/bench_C2.err || { tail -20 $O/bench_C2.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_C2.json').read().strip().splitlines()[-1]); r=d['roofline']; print('C2 auto', round(d['value']/1e6,3), 'M', round(d['ms_per_step']*1e3,1), 'us/step', 'frac', round(r['frac'],4), d['config']['graph']['skewed'])"
