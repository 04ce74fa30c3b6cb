#!/bin/bash
# round 4: slot repair decisions with untimed warm-up cycles before the slot timing
# (FFMP_SLOT_WARMUP) and a tighter slow-slot threshold (FFMP_SLOW_SLOT), C3 bench in fresh processes,
# variants alternating; every timed raster launch dumped (per-slot means of the timed loop)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04h
mkdir -p $O
for rep in 0 1 2; do
  for v in "0 1.12" "2 1.12" "2 1.05"; do
    set -- $v
    tag=w$1_s$2_$rep
    FFMP_SLOT_WARMUP=$1 FFMP_SLOW_SLOT=$2 timeout -k 10 300 python $R/bench.py --steps 40 --warmup 8 --strong-config none --compact-steps 0 --cpu-seconds 0 --dump-launches > $O/$tag.json 2> $O/$tag.err || exit 1
    python -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag', round(d['value']/1e6,3), round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), d['construct_s'], [h.get('slow') for h in d['raster_autotune']['ring']['repair']])"
  done
done
