#!/bin/bash
# round 4: where the env kernel's remaining time goes after the disc-major lidar (every variant of
# tools/env_kernel_breakdown.py at C3 + SQ counters), and the lidar parity suites on the cleaned source
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04d
mkdir -p $O
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_lidar_adversarial.py $R/tests/test_gpu_oracle_c.py -m gpu -x -q --timeout 250 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python $R/tools/env_kernel_breakdown.py --preset C3 --envs 32768 > $O/env_breakdown.txt 2>&1 || exit 1
timeout -k 10 300 python $R/tools/env_kernel_breakdown.py --preset C2 --envs 4096 > $O/env_breakdown_c2.txt 2>&1 || exit 1
timeout -k 10 200 bash $R/tools/gpu_env_pmc.sh > $O/env_pmc.txt 2>&1 || exit 1
