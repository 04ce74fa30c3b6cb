#!/bin/bash
# Round 5: the skewed step graph with the env blocks spread over the first half of the launch: graph parity,
# then C2 / C3 bench with skew (span 0.5, the default), skew with spans 0.25 / 0.9 (probe builds), and serial.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05s
mkdir -p $O
cd $R && timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_graph.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
echo "graph tests: $(tail -1 $O/pytest.log)"
cd /tmp && export TMPDIR=/tmp
for k in 1 2; do
  for cfg in C2 C3; do
    for v in s50 s25 s90 serial; do
      L=$R/flow_field_based_motion_planner_amd/lib/libffmp.so; SK=1
      [ $v = s25 ] && L=$R/tools/_probe/libffmp_span25.so
      [ $v = s90 ] && L=$R/tools/_probe/libffmp_span90.so
      [ $v = serial ] && SK=0
      FFMP_LIB=$L FFMP_GRAPH_SKEW=$SK timeout -k 10 300 python3 $R/bench.py --config $cfg --steps 96 --warmup 16 --cpu-seconds 0 --strong-config none --compact-steps 0 > $O/bench_${cfg}_${v}_$k.json 2> $O/bench_${cfg}_${v}_$k.err || { tail -20 $O/bench_${cfg}_${v}_$k.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/bench_${cfg}_${v}_$k.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$cfg $v', round(d['value']/1e6,2), 'M', round(d['ms_per_step']*1e3,1), 'us/step', 'frac', round(r['frac'],4), round(d['hbm_roofline_pct_whole_step'],2))"
    done
  done
done
