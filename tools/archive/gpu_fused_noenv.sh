#!/bin/bash
# diagnostic: the one-launch step with its env phase removed (tools/_build/libffmp_noenv.so: wave 0
# skips env_group, the raster reads the record from HBM) against the real one-launch step and the
# two-launch step, alternating, C3 bench workload (timing only: the noenv build's envs never move)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
S="import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('%.3f M' % (d['value']/1e6), 'step %.4f' % d['ms_per_step'], r['kernel'], '%.4f ms' % r['kernel_ms'], 'frac %.3f' % r['frac'])"
for k in 1 2; do
  for v in base noenv; do
    if [ $v = base ]; then L=$R/flow_field_based_motion_planner_amd/lib/libffmp.so; else L=$R/tools/_build/libffmp_$v.so; fi
    FFMP_LIB=$L timeout -k 10 300 python3 $R/bench.py --fused on --cpu-seconds 0 --compact-steps 0 > $R/gpurun_out/fne_$v.log 2>&1 || { tail -20 $R/gpurun_out/fne_$v.log; exit 1; }
    echo -n "$v fused: "; grep '^{' $R/gpurun_out/fne_$v.log | python3 -c "$S" || exit 1
  done
  timeout -k 10 300 python3 $R/bench.py --fused off --cpu-seconds 0 --compact-steps 0 > $R/gpurun_out/fne_two.log 2>&1 || exit 1
  echo -n "base two-launch: "; grep '^{' $R/gpurun_out/fne_two.log | python3 -c "$S" || exit 1
done
