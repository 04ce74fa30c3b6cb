#!/bin/bash
# round 3 (second session): the whole GPU suite as the driver runs it, then smoke()
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03b_pytest_gpu.log 2>&1 || { tail -5 gpurun_out/r03b_pytest_gpu.log; grep -E "^E " gpurun_out/r03b_pytest_gpu.log | head -20; exit 1; }
tail -3 gpurun_out/r03b_pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2
