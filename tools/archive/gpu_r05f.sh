#!/bin/bash
# round 5: samples-as-M data gradient variants (tools/_probe): nw4 = 4 waves x 18 positions (one wave per SIMD);
# earlier passes of this script: one k-step per phase with A fragments requested
# up front (kq1up1) or per position (kq1up0), against the shipped two k-steps (ship) and the first version
# (prev); float64 parity of each, then conv2's data gradient at B = 256 / 1024, two alternating passes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05f
mkdir -p $O
for v in ship nw4; do
  lib=$R/flow_field_based_motion_planner_amd/lib/libffmp.so; [ $v = ship ] || lib=$R/tools/_probe/libffmp_$v.so
  FFMP_LIB=$lib timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread $R/tests/test_gpu_conv_mfma.py -k "dgrad_samples_as_m_matches" > $O/pytest_$v.log 2>&1 || { tail -40 $O/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 $O/pytest_$v.log)"
done
for pass in 0 1; do
for v in ship prev nw4; do
  lib=$R/flow_field_based_motion_planner_amd/lib/libffmp.so; [ $v = ship ] || lib=$R/tools/_probe/libffmp_$v.so
  FFMP_LIB=$lib timeout -k 10 300 python $R/tools/conv_probe.py 256 1024 --mfma-only 2>&1 | grep "dgrad bm" | sed "s/^/$v /" || exit 1
done
done
