#!/bin/bash
# round 4: several discs per lane in env_kernel (8 / 16 envs per wave): parity of every layout, whole-config
# C-oracle parity with 8 lanes x 2 discs, then the env kernel alone per layout (FFMP_ENV_LANES)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04k
mkdir -p $O
timeout -k 10 300 python -u -m pytest "$R/tests/test_gpu_parity.py::test_env_lanes_identical" -m gpu -x -q --timeout 250 --timeout-method thread > $O/pytest_lanes.log 2>&1 || { tail -30 $O/pytest_lanes.log; exit 1; }
echo "lanes parity: $(tail -1 $O/pytest_lanes.log)"
FFMP_ENV_LANES=8 timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_oracle_c.py $R/tests/test_gpu_lidar_adversarial.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_l8.log 2>&1 || { tail -30 $O/pytest_l8.log; exit 1; }
echo "8 lanes x 2 discs, oracle parity: $(tail -1 $O/pytest_l8.log)"
for rep in 0 1; do
  for l in 16 8 4; do
    FFMP_ENV_LANES=$l timeout -k 10 200 python $R/tools/env_kernel_breakdown.py --preset C3 --envs 32768 base "L=0 (no lidar)" "no resets" 2>&1 | grep 'env kernel' | sed "s/^/lanes $l /" || exit 1
  done
  # the same 8 x 2 layout held to 4 waves per SIMD (-DFFMP_ENV_WPE=4: 128 VGPRs, 10 spilled), and
  # 16 x 1 held to 5 / 6 waves per SIMD (-DFFMP_ENV_WPE=5 / 6: 96 / 80 VGPRs, 12 / 28 spilled)
  FFMP_LIB=$R/tools/_build/libffmp_wpe4.so FFMP_ENV_LANES=8 timeout -k 10 200 python $R/tools/env_kernel_breakdown.py --preset C3 --envs 32768 base 2>&1 | grep 'env kernel' | sed "s/^/lanes 8 wpe4 /" || exit 1
  for w in 5 6; do
    FFMP_LIB=$R/tools/_build/libffmp_wpe$w.so timeout -k 10 200 python $R/tools/env_kernel_breakdown.py --preset C3 --envs 32768 base 2>&1 | grep 'env kernel' | sed "s/^/lanes 16 wpe$w /" || exit 1
  done
done
for l in 32 16 8; do
  FFMP_ENV_LANES=$l timeout -k 10 200 python $R/tools/env_kernel_breakdown.py --preset C5 --envs 16384 base 2>&1 | grep 'env kernel' | sed "s/^/lanes $l /" || exit 1
done
for l in 16 8; do
  FFMP_ENV_LANES=$l timeout -k 10 200 python $R/tools/env_kernel_breakdown.py --preset C2 --envs 4096 base 2>&1 | grep 'env kernel' | sed "s/^/lanes $l /" || exit 1
done
