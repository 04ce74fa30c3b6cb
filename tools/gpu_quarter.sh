#!/bin/bash
set -o pipefail
hipcc --offload-arch=gfx950 -O3 -o /tmp/quarter_probe tools/quarter_probe.hip > /dev/null 2>&1 || exit 1
timeout -k 10 300 /tmp/quarter_probe 8 2>&1 | grep -v amdgpu.ids
