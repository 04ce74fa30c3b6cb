#!/bin/bash
# round 4: the disc-major lidar (trace_discs) in the shipped lib: env-step parity suites, then the env
# kernel alone against the earlier builds (tools/_build: A = round-3 env_group, N = round-4 env_group
# with the chunked lidar), then the driver's bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04c
mkdir -p $O
B=$R/tools/_build
timeout -k 10 600 python -u -m pytest $R/tests/test_gpu_oracle_c.py $R/tests/test_gpu_parity.py $R/tests/test_spec_geometry.py $R/tests/test_gpu_legacy_api.py $R/tests/test_gpu_ros_bridge.py $R/tests/test_gpu_lidar_adversarial.py -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 0 1; do
  for v in A N main; do
    L=$B/libffmp_$v.so; [ $v = main ] && L=$R/flow_field_based_motion_planner_amd/lib/libffmp.so
    FFMP_LIB=$L timeout -k 10 200 python3 $R/tools/env_kernel_breakdown.py --preset C3 --envs 32768 base "L=0 (no lidar)" 2>&1 | grep 'env kernel' | sed "s/^/$v /" || exit 1
  done
done
for v in A N main; do
  L=$B/libffmp_$v.so; [ $v = main ] && L=$R/flow_field_based_motion_planner_amd/lib/libffmp.so
  FFMP_LIB=$L timeout -k 10 200 python3 $R/tools/env_kernel_breakdown.py --preset C5 --envs 16384 base 2>&1 | grep 'env kernel' | sed "s/^/$v /" || exit 1
done
timeout -k 10 400 python $R/bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 1
