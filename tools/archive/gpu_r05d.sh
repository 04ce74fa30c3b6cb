#!/bin/bash
# round 5: the samples-as-M data gradient, B fragments and next-phase pieces over two register sets vs one
# (tools/_probe/libffmp_prev.so: the first version), float64 parity of the shipped build, conv2 at B = 256 / 1024
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05d
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread $R/tests/test_gpu_conv_mfma.py -k "dgrad" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in ship prev ship prev; do
  lib=$R/flow_field_based_motion_planner_amd/lib/libffmp.so; [ $v = ship ] || lib=$R/tools/_probe/libffmp_$v.so
  FFMP_LIB=$lib timeout -k 10 300 python $R/tools/conv_probe.py 256 1024 --mfma-only 2>&1 | grep "dgrad bm" | sed "s/^/$v /" || exit 1
done
