#!/bin/bash
# GPU parity suite on the in-tree lib, then tools/gpu_ab_bench.sh (base vs new).  usage: [reps]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/pytest_gpu.log 2>&1 || { tail -30 $R/gpurun_out/pytest_gpu.log; exit 1; }
tail -1 $R/gpurun_out/pytest_gpu.log
bash $R/tools/gpu_ab_bench.sh ${1:-3}
