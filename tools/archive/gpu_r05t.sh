#!/bin/bash
# Round 5: the skewed graph in bench.py (auto: both graphs timed, the faster kept) and in the full-size timed
# path: graph tests, the timed path (f32 incl. skewed graph replays, u8f16), bench C2 / C3 twice.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05t
mkdir -p $O
export FFMP_TIMED_PATH_OUT=$O
cd $R && timeout -k 10 900 python3 -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu tests/test_gpu_graph.py tests/test_gpu_timed_path.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
echo "tests: $(tail -1 $O/pytest.log)"
cd /tmp && export TMPDIR=/tmp
for k in 1 2; do
  for cfg in C2 C3; do
    timeout -k 10 400 python3 $R/bench.py --config $cfg --steps 96 --warmup 16 --cpu-seconds 0 --strong-config none --compact-steps 0 > $O/bench_${cfg}_$k.json 2> $O/bench_${cfg}_$k.err || { tail -20 $O/bench_${cfg}_$k.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/bench_${cfg}_$k.json').read().strip().splitlines()[-1]); r=d['roofline']; g=d['config']['graph']; print('$cfg', round(d['value']/1e6,2), 'M', round(d['ms_per_step']*1e3,1), 'us/step', 'frac', round(r['frac'],4), round(d['hbm_roofline_pct_whole_step'],2), 'skewed', g['skewed'], g['skew_trial'])"
  done
done
