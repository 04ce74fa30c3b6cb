#!/bin/bash
# Round 5: the skewed graph at C3 with the env step on at most P env blocks (each stepping several blocks' worth
# of envs in turn; FFMP_SKEW_ENV_BLOCKS, default = the CU count): P = 128 / 256 / 512 / 2048 against the
# two-launch graph, alternating, two rounds; then the graph tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05u
mkdir -p $O
cd $R && timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_graph.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
echo "graph tests: $(tail -1 $O/pytest.log)"
cd /tmp && export TMPDIR=/tmp
for k in 1 2; do
  for v in 128 256 512 2048 off; do
    SK=on; [ $v = off ] && SK=off
    FFMP_SKEW_ENV_BLOCKS=$v timeout -k 10 300 python3 $R/bench.py --config C3 --graph-skew $SK --steps 96 --warmup 16 --cpu-seconds 0 --strong-config none --compact-steps 0 > $O/bench_${v}_$k.json 2> $O/bench_${v}_$k.err || { tail -20 $O/bench_${v}_$k.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/bench_${v}_$k.json').read().strip().splitlines()[-1]); r=d['roofline']; print('C3 env blocks $v', round(d['value']/1e6,3), 'M', round(d['ms_per_step']*1e3,1), 'us/step', 'frac', round(r['frac'],4), round(d['hbm_roofline_pct_whole_step'],2))"
  done
done
