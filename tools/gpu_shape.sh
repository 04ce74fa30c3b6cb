#!/bin/bash
set -o pipefail
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > /dev/null 2>&1 || exit 1
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x -k "raster_parity or odd_sizes" 2>&1 | tail -1
for c in C3 C5 C2; do timeout -k 10 300 python tools/raster_shape_ab.py $c 5 2>&1 | grep -v amdgpu.ids || exit 1; done
