#!/bin/bash
# round 5 baseline on a fresh box: the driver's bench line, C2 at 200 steps, the learner convolutions at B = 256
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05a
mkdir -p $O
timeout -k 10 400 python $R/bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1]); print('default', round(d['value']/1e6,3), round(d['roofline']['kernel_ms'],4), round(d['roofline']['frac'],4), round(d['hbm_roofline_pct_whole_step'],2), round(d['compact_layout']['value']/1e6,3), round(d['strong']['value']/1e6,3))"
timeout -k 10 300 python $R/bench.py --config C2 --steps 200 --warmup 20 --strong-config none --compact-steps 0 --cpu-seconds 0 > $O/bench_c2.json 2> $O/bench_c2.err || exit 1
python -c "import json; d=json.loads(open('$O/bench_c2.json').read().strip().splitlines()[-1]); print('c2', round(d['value']/1e6,3), round(d['roofline']['kernel_ms'],4), round(d['roofline']['frac'],4), round(d['hbm_roofline_pct_whole_step'],2), d['raster_autotune'].get('fused'))"
timeout -k 10 300 python $R/tools/conv_probe.py 256 --mfma-only > $O/conv_probe.log 2>&1 || { tail -20 $O/conv_probe.log; exit 1; }
cat $O/conv_probe.log
