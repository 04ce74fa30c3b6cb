#!/bin/bash
# round 3 (second session): slow start after reset(): episodes or GPU state (tools/transient_reset.py)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/transient_reset.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r03b_transient_reset.txt
