#!/bin/bash
# C2 with partner relocation allowed (RELOCATE_MIN_BYTES) vs the previous threshold (4 GiB:
# FFMP_TEST_NO_RELOC=1 restores it), alternating fresh processes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/c2r
for rep in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then X="import flow_field_based_motion_planner_amd.vec_env as m; m.FFMPVec.RELOCATE_MIN_BYTES = 4 << 30"; else X="pass"; fi
    timeout -k 10 200 python3 -c "$X
import runpy, sys; sys.argv = ['bench.py', '--config', 'C2', '--steps', '100', '--warmup', '10', '--cpu-seconds', '0', '--compact-steps', '0']; runpy.run_path('$R/bench.py', run_name='__main__')" > $R/gpurun_out/c2r/b.log 2>&1 || { tail -5 $R/gpurun_out/c2r/b.log; exit 1; }
    grep '^{' $R/gpurun_out/c2r/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; g=d['raster_autotune'].get('ring', {}); print('$v', round(d['value']/1e6,2), 'M', r['kernel'], round(r['kernel_ms'],4), round(r['achieved']), 'GB/s', g.get('pair_gbs_max'), g.get('partner_tries'))" || exit 1
  done
done
