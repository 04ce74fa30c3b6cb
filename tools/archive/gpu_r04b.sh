#!/bin/bash
# round 4: lidar variants (tools/gpu_r04_lidar.sh), step_many parity, bench C3 / C2 with the open-loop leg
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04b
mkdir -p $O
bash $R/tools/gpu_r04_lidar.sh > $O/lidar.txt 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread $R/tests/test_gpu_step_many.py > $O/pytest_step_many.log 2>&1 || exit 1
timeout -k 10 400 python $R/bench.py --steps 20 --warmup 5 > $O/bench_c3.json 2> $O/bench_c3.err || exit 1
timeout -k 10 300 python $R/bench.py --config C2 --steps 200 --warmup 20 --strong-config none --compact-steps 0 --cpu-seconds 0 > $O/bench_c2.json 2> $O/bench_c2.err || exit 1
