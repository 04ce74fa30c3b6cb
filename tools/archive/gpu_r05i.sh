#!/bin/bash
# Round 5: compact raster (u8f16) with the per-column-band cull terms (no spill reloads in the band
# loop) against HEAD's kernel (tools/_probe/libffmp_prev.so), 3 alternating rounds, then the
# compact parity tests on the new library.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05i
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for k in 1 2 3; do
  for v in new prev; do
    L=$R/flow_field_based_motion_planner_amd/lib/libffmp.so
    [ $v = prev ] && L=$R/tools/_probe/libffmp_prev.so
    echo "== $v round $k"
    FFMP_LIB=$L timeout -k 10 180 python3 $R/bench.py --obs-format u8f16 --steps 40 --warmup 5 --cpu-seconds 0 > $O/bench_${v}_$k.json 2> $O/bench_${v}_$k.err || exit 1
    python3 -c "import json,sys; d=json.loads(open('$O/bench_${v}_$k.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['roofline']['frac'], d['roofline']['achieved'])"
  done
done
echo "== shapes new"
timeout -k 10 180 python3 $R/tools/compact_shapes.py C3 u8f16 > $O/shapes_new.txt 2>&1 || exit 1
cat $O/shapes_new.txt
echo "== tests"
cd $R && timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_compact.py tests/test_gpu_timed_path.py > $O/pytest.log 2>&1; s=$?; tail -5 $O/pytest.log; exit $s
