#!/bin/bash
# Round 5: the ring's pairing acceptance (a piece is taken when its two-stream probe is within the factor of the best
# seen; 0.93 by default) at 0.97 / 0.985 (probe builds), compact layout C3 (1:2 stores) and f32 C3, alternating.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05z
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for k in 1 2; do
  for fmt in u8f16 f32; do
    for v in base pa97 pa985; do
      L=$R/flow_field_based_motion_planner_amd/lib/libffmp.so
      [ $v != base ] && L=$R/tools/_probe/libffmp_$v.so
      FFMP_LIB=$L timeout -k 10 300 python3 $R/bench.py --obs-format $fmt --steps 48 --warmup 8 --cpu-seconds 0 --strong-config none --compact-steps 0 > $O/b_${fmt}_${v}_$k.json 2> $O/b_${fmt}_${v}_$k.err || { tail -20 $O/b_${fmt}_${v}_$k.err; exit 1; }
      python3 -c "
import json; d=json.loads(open('$O/b_${fmt}_${v}_$k.json').read().strip().splitlines()[-1]); ra=d['raster_autotune']; ri=ra['ring']; sm=ri['repair'][-1]['slot_ms']
print('$fmt $v', round(d['value']/1e6,3), 'M frac', round(d['roofline']['frac'],4), 'raster gbs', ra['gbs'], 'pairs', ri['pair_gbs_min'], ri['pair_gbs_max'], 'probes', ri['pair_probes'], 'slot mean', round(sum(sm)/len(sm),4), 'construct', d['construct_s'])"
    done
  done
done
