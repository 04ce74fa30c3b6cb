#!/bin/bash
# round 4: the ring's pairing budget (one extra fresh piece per position) + slot timing after two
# warm-up cycles + a 6 % slow-slot threshold: the C3 bench in fresh processes, timed launches dumped
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04i
mkdir -p $O
for rep in 0 1 2 3 4 5; do
  tag=run$rep
  timeout -k 10 300 python $R/bench.py --steps 40 --warmup 8 --strong-config none --compact-steps 0 --cpu-seconds 0 --dump-launches > $O/$tag.json 2> $O/$tag.err || exit 1
  python -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); r=d['raster_autotune']['ring']; print('$tag', round(d['value']/1e6,3), round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), d['construct_s'], r.get('pieces_new'), r.get('pair_gbs_min'), [h.get('slow') for h in r['repair']], r.get('reverts'))"
done
python $R/tools/slot_means.py 8 $O/run*.err
timeout -k 10 400 python $R/bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || exit 1
python -c "import json; d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1]); print('default', round(d['value']/1e6,3), round(d['roofline']['kernel_ms'],4), d['construct_s'], round(d['compact_layout']['value']/1e6,3), round(d['strong']['value']/1e6,3))"
