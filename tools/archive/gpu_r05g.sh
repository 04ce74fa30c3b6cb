#!/bin/bash
# round 5: HIP-graph replay of whole steps (FFMPVec.capture): parity, then C2 (200 steps) eager and graph, twice
# each on one box, and the default C3 line with --graph on (C2 with the 8-round one-/two-launch recheck)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05g
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread $R/tests/test_gpu_graph.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 0 1; do
for g in off on; do
  timeout -k 10 300 python $R/bench.py --config C2 --steps 200 --warmup 20 --strong-config none --compact-steps 0 --cpu-seconds 0 --graph $g > $O/c2_${g}_$rep.json 2> $O/c2_${g}_$rep.err || { tail -20 $O/c2_${g}_$rep.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/c2_${g}_$rep.json').read().strip().splitlines()[-1]); f=d['raster_autotune'].get('fused') or {}; print('c2 graph=$g', round(d['value']/1e6,3), 'M', round(d['ms_per_step'],4), 'ms/step', d['roofline']['kernel'], round(d['roofline']['kernel_ms'],4), round(d['roofline']['frac'],4), round(d['hbm_roofline_pct_whole_step'],2), 'fused', d['config']['fused'], (f.get('recheck') or {}).get('two_launch_step_ms'), (f.get('recheck') or {}).get('fused_step_ms'))"
done
done
timeout -k 10 400 python $R/bench.py --steps 24 --warmup 8 --graph on --compact-steps 0 --cpu-seconds 0 --strong-config none > $O/c3_graph.json 2> $O/c3_graph.err || { tail -20 $O/c3_graph.err; exit 1; }
python -c "import json; d=json.loads(open('$O/c3_graph.json').read().strip().splitlines()[-1]); print('c3 graph', round(d['value']/1e6,3), 'M', round(d['ms_per_step'],4), d['roofline']['kernel'], round(d['roofline']['kernel_ms'],4), round(d['roofline']['frac'],4), round(d['hbm_roofline_pct_whole_step'],2), 'fused', d['config']['fused'])"
timeout -k 10 400 python $R/bench.py --steps 24 --warmup 8 --compact-steps 0 --cpu-seconds 0 --strong-config none > $O/c3_eager.json 2> $O/c3_eager.err || { tail -20 $O/c3_eager.err; exit 1; }
python -c "import json; d=json.loads(open('$O/c3_eager.json').read().strip().splitlines()[-1]); print('c3 eager', round(d['value']/1e6,3), 'M', round(d['ms_per_step'],4), d['roofline']['kernel'], round(d['roofline']['kernel_ms'],4), round(d['roofline']['frac'],4), round(d['hbm_roofline_pct_whole_step'],2), 'fused', d['config']['fused'])"
