#!/bin/bash
# Round 5: C2 in graph replays — one-launch step (fused on) vs two-launch (serial graph), alternating.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05o
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for k in 1 2; do
  for f in on off; do
    FFMP_GRAPH_PIPELINE=0 timeout -k 10 300 python3 $R/bench.py --config C2 --fused $f --steps 96 --warmup 16 --cpu-seconds 0 --strong-config none --compact-steps 0 > $O/c2_f${f}_$k.json 2> $O/c2_f${f}_$k.err || { tail -20 $O/c2_f${f}_$k.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/c2_f${f}_$k.json').read().strip().splitlines()[-1]); r=d['roofline']; print('C2 fused=$f', round(d['value']/1e6,2), 'M', round(d['ms_per_step']*1e3,1), 'us/step', 'frac', round(r['frac'],4), r.get('kernel'))"
  done
done
