#!/bin/bash
# Round 5: the skewed step graph (raster of step i + env step of step i + 1 in ONE launch, ffmp_step_skewed):
# graph parity tests, then bench.py C2 and C3 with the skewed graph (default) and the serial graph
# (FFMP_GRAPH_SKEW=0), alternating, two rounds each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05r
mkdir -p $O
cd $R && timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_graph.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
echo "graph tests: $(tail -1 $O/pytest.log)"
cd /tmp && export TMPDIR=/tmp
for k in 1 2; do
  for cfg in C2 C3; do
    for p in 1 0; do
      FFMP_GRAPH_SKEW=$p timeout -k 10 300 python3 $R/bench.py --config $cfg --steps 96 --warmup 16 --cpu-seconds 0 --strong-config none --compact-steps 0 > $O/bench_${cfg}_s${p}_$k.json 2> $O/bench_${cfg}_s${p}_$k.err || { tail -20 $O/bench_${cfg}_s${p}_$k.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/bench_${cfg}_s${p}_$k.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$cfg skew=$p', round(d['value']/1e6,2), 'M', round(d['ms_per_step']*1e3,1), 'us/step', 'frac', round(r['frac'],4), round(d['hbm_roofline_pct_whole_step'],2))"
    done
  done
done
