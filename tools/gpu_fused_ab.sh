#!/bin/bash
# one-launch step change: GPU parity suite, fused-kernel phase trace, alternating bench A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/pytest_gpu.log 2>&1 || { tail -30 $R/gpurun_out/pytest_gpu.log; exit 1; }
tail -1 $R/gpurun_out/pytest_gpu.log
FFMP_LIB=$R/tools/_build/libffmp_trace.so timeout -k 10 300 python3 $R/tools/trace_probe.py C3 32768 fused 2>&1 | grep -v amdgpu.ids | head -6 || exit 1
bash $R/tools/gpu_ab_bench.sh ${1:-3}
