#!/bin/bash
# round 3 (second session): the post-idle slow start by raster launch shape (tools/transient_shapes.py)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/transient_shapes.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r03b_transient_shapes.txt
